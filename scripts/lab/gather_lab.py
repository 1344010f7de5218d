#!/usr/bin/env python3
"""Lab (not product): rank gather of one endpoint over records in stream order vs records
partitioned by that endpoint's top bits, with and without XCD-contiguous tile mapping."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from sheep_amd import device  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 26
lab = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libedgelab.so"))
device.init(0)
uv = device.rmat(S, 16, S)
deg = device.degree(uv, 1 << S)
seq, rank, n_seq = device.sequence(deg)
m = uv.shape[0]
out = torch.empty(m, dtype=torch.int64, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for name, recs in [("stream order", uv)]:
    for xcd in (0, 1):
        ms = timeit(lambda: lab.gather_lab(xcd, P(recs), ctypes.c_uint64(m), P(rank), P(out), st))
        print("%-28s xcd=%d  %.3f ms" % (name, xcd, ms), flush=True)
y = uv.view(torch.int32)[:, 1].to(torch.int64) & 0xFFFFFFFF
for bits in (8, 10, 12):
    key = y >> (S - bits)
    order = torch.argsort(key, stable=True)
    recs = uv.view(torch.int64)[order].contiguous().view(torch.uint32).view(-1, 2)
    del order
    for xcd in (0, 1):
        ms = timeit(lambda: lab.gather_lab(xcd, P(recs), ctypes.c_uint64(m), P(rank), P(out), st))
        print("%-28s xcd=%d  %.3f ms" % ("partitioned by y top %d b" % bits, xcd, ms), flush=True)
    del recs
