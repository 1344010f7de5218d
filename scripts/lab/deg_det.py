"""Determinism of the degree pass of a given library build (lab check): twitter-shape records,
three passes per option set."""
import sys
import torch

from sheep_amd import capi, device

if len(sys.argv) > 1:
    capi.lib_path = sys.argv[1]

device.init(0)
uv = device.powerlaw(41652230, 1468365182, 2.1, 50.0, 5)
torch.cuda.synchronize()
for plain in (1, 0):
    capi.set_option("degb_plain", plain)
    ref, out = None, []
    for rep in range(3):
        d = device.degree(uv, 41652230).view(torch.int32).to(torch.int64)
        torch.cuda.synchronize()
        ref = d if ref is None else ref
        out.append((int(d.sum()), int((d != ref).sum())))
    print(sys.argv[1:], "plain", plain, out, flush=True)
