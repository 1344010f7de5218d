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


@pytest.mark.gpu
def test_rmat27_beyond_u32_endpoints(gpu):
    """R-MAT scale 27: 2^31 records, 2^32 endpoints — past round 2's u32 endpoint offsets (the
    fused degree pass counts records, so one GPU takes m < 2^32).  Checked without a CPU run,
    by properties that hold at any size:
      * the whole stream's degrees equal the sum of its two halves' (each half on the bucketed
        endpoint path, within the old limits);
      * the whole stream's tree equals the exact merge of the two halves' trees, each built on
        the global seq (etree(G1 ∪ G2) = etree(etree(G1) ∪ etree(G2)); pst summed: the merge of
        jnode.cpp:174-201, what graph2tree -l + merge_trees relies on, README:112-121)."""
    import torch

    from sheep_amd import device

    scale, n_ids = 27, 1 << 27
    uv = device.rmat(scale, 16, 27)
    m = uv.shape[0]
    assert 2 * m == 1 << 32
    seq, parent, pst, n = device.graph2tree(uv, n_ids)
    deg, _ = device.degree_ex(uv, n_ids)
    h = m // 2
    d0, s0 = device.degree_ex(uv[:h], n_ids)
    d1, s1 = device.degree_ex(uv[h:], n_ids)
    torch.cuda.synchronize()
    i32 = lambda t: t.view(torch.int32)  # noqa: E731 (u32 add = i32 add, two's complement)
    assert torch.equal(i32(deg), i32(d0) + i32(d1))
    seq2, rank, n2 = device.sequence(deg)
    assert n2 == n and torch.equal(i32(seq2[:n]), i32(seq[:n]))
    pa, wa = device.build_tree_deg(uv[:h], rank, seq2, n, d0, s0)
    pb, wb = device.build_tree_deg(uv[h:], rank, seq2, n, d1, s1)
    device.merge_into(pa, wa, pb, wb, n)
    torch.cuda.synchronize()
    assert torch.equal(i32(pa[:n]), i32(parent[:n]))
    assert torch.equal(i32(wa[:n]), i32(pst[:n]))
    # and the forest is heap-ordered (parent > child, INVALID at the roots)
    p = parent[:n].to(torch.int64) & 0xFFFFFFFF
    idx = torch.arange(n, device=p.device)
    assert bool(((p == 0xFFFFFFFF) | (p > idx)).all())
