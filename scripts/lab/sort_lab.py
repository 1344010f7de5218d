#!/usr/bin/env python3
"""Lab (not product): hipCUB radix sort time on the edge items of R-MAT (speed reference)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from sheep_amd import device  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 26
here = os.path.dirname(os.path.abspath(__file__))
lab = ctypes.CDLL(os.path.join(here, "libedgelab.so"))
srt = ctypes.CDLL(os.path.join(here, "libsortlab.so"))
device.init(0)
uv = device.rmat(S, 16, S)
deg = device.degree(uv, 1 << S)
seq, rank, n_seq = device.sequence(deg)
m = uv.shape[0]
items = torch.empty(m, dtype=torch.int64, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())
assert lab.edge_lab(0, P(uv), ctypes.c_uint64(m), P(rank), None, P(items), 2048, 256, st) == 0
del uv
out = torch.empty_like(items)
top = n_seq.bit_length()
for lo_bit in (32, 32 + top - 16, 32 + top - 8):
    tb = ctypes.c_size_t(0)
    assert srt.sort_lab(P(items), P(out), ctypes.c_uint64(m), lo_bit, 32 + top + 1, None, ctypes.byref(tb), st) == 0
    tmp = torch.empty(tb.value, dtype=torch.uint8, device="cuda")
    def run():
        assert srt.sort_lab(P(items), P(out), ctypes.c_uint64(m), lo_bit, 32 + top + 1, P(tmp), ctypes.byref(tb), st) == 0
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print("hipcub SortKeys u64 n=%d bits [%d,%d): %.3f ms (%d passes of 8 b at ~%.2f ms)" % (
        m, lo_bit, 32 + top + 1, ms, (32 + top + 1 - lo_bit + 7) // 8, ms / ((32 + top + 1 - lo_bit + 7) // 8)), flush=True)
    del tmp
