"""Full-size parity at the BASELINE.json configs (C2 RMAT-22, C3 LJ-shape, C4 RMAT-26, C5
twitter-shape) against the CPU checker's committed digests (tests/golden/digests.json, made by
tests/golden/make_digests.py in the build container: the checker needs minutes per config, the
GPU seconds).

Per config, on cuda:0 through the C-ABI:
  * sheep_graph2tree_dev (degree -> sequence -> tree, LLAMA degrees): n_seq and SHA-256 of
    seq / parent / pst_weight equal the checker's (jtree.cpp:65-145 bit-exact);
  * the 8-GPU driver (per-shard degrees summed, per-shard maps, every shard's kept pairs applied
    by all; sheep_graph2tree_multi_local = the C++ loop of sheep_graph2tree_multi_dev with its
    collectives as device copies) with 8 rank threads on one device: same hashes;
  * sheep_partition (the product's host forwardPartition, partition.cpp:50-157) on the GPU tree
    for k = 16, 64, 256 on one table, then sheep_evaluate_dev (partition.cpp:428-521): the
    parts hash, the part count and every evaluate number (edges cut, Vcom vol, ECV(hash/down/
    up) and their balances) equal the checker's.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

DIGESTS = json.load(open(os.path.join(GOLDEN, "digests.json")))
NAMES = sorted(k for k in DIGESTS if not k.startswith("_"))
INV = 0xFFFFFFFF


def h16(t):
    a = t.cpu().numpy() if hasattr(t, "cpu") else t
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8)).hexdigest()[:16]


def records(spec, lo=0, hi=None):
    from sheep_amd import device

    if spec["kind"] == "rmat":
        return device.rmat(spec["scale"], spec["edgefactor"], spec["seed"], lo, hi)
    return device.powerlaw(spec["n"], spec["m"], spec["gamma"], spec["i0"], spec["seed"], lo, hi)


def u32(t, n):
    import torch

    return t[:n].view(torch.int32).cpu().numpy().view(np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_fullsize_tree_and_partition(gpu, name):
    import torch

    from sheep_amd import api, device

    d = DIGESTS[name]
    uv = records(d)
    assert uv.shape[0] == d["records"]
    seq_d, parent_d, pst_d, n = device.graph2tree(uv, d["n_ids"])
    torch.cuda.synchronize()
    assert n == d["n_seq"]
    seq, parent, pst = u32(seq_d, n), u32(parent_d, n), u32(pst_d, n)
    assert (h16(seq), h16(parent), h16(pst)) == (d["seq"], d["parent"], d["pst"])
    # partition on the host (product code), evaluate on the GPU
    ks = [int(k) for k in sorted(d["partition"], key=int)]
    parts, created = api.partition(api.JNodeTable(parent, pst), seq, ks)
    rank = torch.full((d["n_ids"],), -1, dtype=torch.int32, device="cuda")
    rank[seq_d[:n].view(torch.int32).long()] = torch.arange(n, dtype=torch.int32, device="cuda")
    for k, p, c in zip(ks, parts, created):
        want = d["partition"][str(k)]
        assert (h16(p), c) == (want["parts"], want["created"]), k
        full = np.full(d["n_ids"], -1, np.int16)
        full[:p.size] = p
        ev = device.evaluate(uv, torch.from_numpy(full).cuda(), rank.view(torch.uint32), c)
        got = {key: ev[key] for key in device.EVAL_KEYS}
        assert got == {key: want[key] for key in device.EVAL_KEYS}, k
    del uv
    torch.cuda.empty_cache()
    gpu.call("sheep_release")


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_fullsize_8_ranks(gpu, name):
    """The 8-GPU driver (sheep_graph2tree_multi_dev's loop) with 8 shards as 8 rank threads on
    one device: the same tree as the checker's, on every rank."""
    import torch

    from sheep_amd import device
    from sheep_amd.dist import shard_bounds

    d = DIGESTS[name]
    P = 8
    shards = [records(d, *shard_bounds(d["records"], r, P)) for r in range(P)]
    seq_d, parent_d, pst_d, n = device.graph2tree_multi_local(shards, d["n_ids"])
    torch.cuda.synchronize()
    assert n == d["n_seq"]
    assert (h16(u32(seq_d, n)), h16(u32(parent_d, n)), h16(u32(pst_d, n))) == \
        (d["seq"], d["parent"], d["pst"])
    del shards
    torch.cuda.empty_cache()
    gpu.call("sheep_release")
