#!/usr/bin/env python3
"""Lab (not product): time edge-pass variants on R-MAT in HBM (torch events on the stream)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from sheep_amd import device  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 26
variants = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2, 3, 4, 5, 6, 7, 8]
lab = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libedgelab.so"))
device.init(0)
uv = device.rmat(S, 16, S)
deg = device.degree(uv, 1 << S)
seq, rank, n_seq = device.sequence(deg)
m = uv.shape[0]
items = torch.empty(m, dtype=torch.int64, device="cuda")
r3 = torch.zeros(3 * (1 << S) + 64, dtype=torch.uint8, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())
assert lab.edge_lab(100, P(uv), ctypes.c_uint64(1 << S), P(rank), None, P(r3), 0, 0, st) == 0
ref = None
for grid, block in [(2048, 256), (8192, 256), (1024, 1024)]:
    for v in variants:
        def run():
            assert lab.edge_lab(v, P(uv), ctypes.c_uint64(m), P(rank), P(r3), P(items), grid, block, st) == 0
        run()
        torch.cuda.synchronize()
        if v not in (2, 3):
            if ref is None:
                ref = items.clone()
            ok = bool(torch.equal(ref, items))
        else:
            ok = "-"
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print("grid %5d block %4d variant %3d  %.3f ms  %.1f GB/s(16B/e)  same=%s" % (
            grid, block, v, ms, 16 * m / ms / 1e6, ok), flush=True)
