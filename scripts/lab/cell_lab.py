#!/usr/bin/env python3
"""Lab (not product): rank-gather cost by record order (scripts/lab/cell_lab.hip), RMAT-S:
one endpoint from records partitioned by its top 8 bits (today's part<1> / edge pass) vs
both endpoints from records partitioned into 2D (y, x) cells of 2^c x 2^c."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from sheep_amd import device  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 26
lab = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcelllab.so"))
device.init(0)
uv = device.rmat(S, 16, S)
deg = device.degree(uv, 1 << S)
seq, rank, n_seq = device.sequence(deg)
del deg, seq
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


w = uv.view(torch.int64)
x = w & 0xFFFFFFFF
y = (w >> 32) & 0xFFFFFFFF


def ordered(key):
    """Records grouped by key value (<= 256 values; torch.argsort is not used: over 2^30
    elements it returned a wrong permutation here), checked to be a permutation."""
    parts = [w[key == d] for d in range(int(key.max()) + 1)]
    r = torch.cat(parts)
    del parts
    assert r.numel() == m and int(r.sum()) == int(w.sum()) and int((r & 0xFFFF).sum()) == int((w & 0xFFFF).sum())
    return r.view(torch.uint32).view(-1, 2)


def run(name, recs, mode):
    for xcd in (0, 1):
        ms = timeit(lambda: lab.cell_lab(mode, xcd, P(recs), ctypes.c_uint64(m), P(rank), P(out), st))
        print("%-34s xcd=%d %7.3f ms" % (name, xcd, ms), flush=True)


degt = torch.zeros(1 << S, dtype=torch.int32, device="cuda")


def rund(name, recs):
    for xcd in (0, 1):
        ms = timeit(lambda: lab.deg_lab(xcd, P(recs), ctypes.c_uint64(m), P(degt), st))
        print("%-34s xcd=%d %7.3f ms" % (name, xcd, ms), flush=True)


run("stream order, both", uv, 2)
run("stream order, copy", uv, 3)
r = ordered(y >> (S - 8)); run("y top 8, rank[y]", r, 0); del r
r = ordered(x >> (S - 8)); run("x top 8, rank[x]", r, 1); del r
for c in (1, 2, 3, 4):
    r = ordered(((y >> (S - c)) << c) | (x >> (S - c)))
    run("cells %dx%d, both" % (1 << c, 1 << c), r, 2)
    del r
rund("stream order, degree atomics", uv)
