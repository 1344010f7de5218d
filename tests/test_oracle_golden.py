"""The CPU checker (oracle/) pinned against the reference's own published fixtures.

hep-th: data/hep-th.dat with the TREEFAQS digest and the partition_tree -f -g output for
k = 2..32 published in data/quality/hep.degree.raw (extracted by tests/golden/make_goldens.py).
Known-answer graph: SURVEY Appendix A7.
"""
import json
import os
import tempfile

import numpy as np
import pytest

from conftest import GOLDEN

PUB = json.load(open(os.path.join(GOLDEN, "hep_th_published.json")))
KA = json.load(open(os.path.join(GOLDEN, "known_answer.json")))


def test_hep_th_records(hep_edges):
    assert hep_edges.shape == (PUB["ini"]["edges"], 2)
    assert int(hep_edges.max()) + 1 == PUB["ini"]["vertices"]


def test_hep_th_treefaqs(oracle, hep_edges):
    seq = oracle.degree_sequence(hep_edges)
    p, s = oracle.build_tree(hep_edges, seq)
    assert oracle.facts(p, s) == PUB["treefaqs"]


def test_hep_th_partitions_all_k(oracle, hep_edges):
    """One partition_tree run over k = 2..32 (kids order persists across k)."""
    seq = oracle.degree_sequence(hep_edges)
    p, s = oracle.build_tree(hep_edges, seq)
    pt = oracle.PartTree(p, s)
    for rec in PUB["partitions"]:
        k = rec["k"]
        parts = pt.partition(seq, k)
        ev = oracle.evaluate(hep_edges, parts, seq)
        assert int(parts.max()) + 1 == rec["created"], k
        assert int((parts == 0).sum()) == rec["size0"], k
        assert int((parts == 1).sum()) == rec["size1"], k
        for key in ("edges_cut", "vcom_vol", "ecv_hash", "ecv_down", "ecv_up"):
            assert ev[key] == rec[key], (k, key)
            assert "%f" % (ev[key] / ev["edges"]) == rec[key + "_pct"], (k, key)


def test_known_answer(oracle):
    uv = np.array(KA["records"], np.uint32)
    seq = oracle.degree_sequence(uv)
    assert seq.tolist() == KA["llama_seq"]
    p, s = oracle.build_tree(uv, seq)
    assert [-1 if x == oracle.INVALID else int(x) for x in p] == KA["parent"]
    assert s.tolist() == KA["pst"]
    assert oracle.facts(p, s) == KA["treefaqs"]
    assert oracle.degree_sequence(uv, oracle.FILE).tolist() == KA["file_seq_stream"]


def test_known_answer_xs1reader_quirk(oracle, tmp_path):
    uv = np.array(KA["records"], np.uint32)
    rec = np.zeros((len(uv), 3), np.uint32)
    rec[:, :2] = uv
    rec[:, 2] = np.float32(1.0).view(np.uint32)
    path = str(tmp_path / "ka.dat")
    rec.tofile(path)
    assert np.array_equal(oracle.read_dat(path), uv)
    stream = oracle.read_dat_xs1reader(path)
    assert len(stream) == len(uv) + 1 and tuple(stream[-1]) == tuple(uv[-1])
    assert oracle.degree_sequence(stream, oracle.FILE).tolist() == KA["file_seq_dat_xs1reader"]


def test_net_reader_stops_at_comment(oracle, tmp_path):
    path = str(tmp_path / "g.net")
    open(path, "w").write("0 1\n2 3\n# comment\n4 5\n")
    assert oracle.read_net(path).tolist() == [[0, 1], [2, 3]]


def is_etree(uv, seq, parent):
    """parent(r) = min{t > r : t adjacent to subtree(r)}, checked by brute force."""
    n = len(seq)
    rank = {int(v): i for i, v in enumerate(seq)}
    adj = [set() for _ in range(n)]
    for a, b in uv:
        if a != b and int(a) in rank and int(b) in rank:
            ra, rb = rank[int(a)], rank[int(b)]
            adj[ra].add(rb)
            adj[rb].add(ra)
    kids = [[] for _ in range(n)]
    for v in range(n):
        if parent[v] != 0xFFFFFFFF:
            kids[int(parent[v])].append(v)
    for r in range(n):
        stack, sub = [r], []
        while stack:
            x = stack.pop()
            sub.append(x)
            stack.extend(kids[x])
        cand = [t for x in sub for t in adj[x] if t > r]
        want = min(cand) if cand else 0xFFFFFFFF
        if int(parent[r]) != want:
            return False
    return True


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_tree_is_etree_small_random(oracle, seed):
    rng = np.random.default_rng(seed)
    uv = rng.integers(0, 60, size=(150, 2)).astype(np.uint32)
    seq = oracle.degree_sequence(uv)
    p, s = oracle.build_tree(uv, seq)
    assert is_etree(uv, seq, p)


def test_oracle_merge_of_shards_equals_whole(oracle):
    """README:112-121: partial loads merged pairwise reproduce the serial tree (-l i/k)."""
    uv = oracle.rmat(12, 16, 7)
    seq = oracle.degree_sequence(uv)
    whole = oracle.build_tree(uv, seq)
    for k in (2, 3, 4):
        R = len(uv)
        trees = [oracle.build_tree(uv[R * i // k: R * (i + 1) // k], seq) for i in range(k)]
        acc = trees[0]
        for t in trees[1:]:
            acc = oracle.merge(acc[0], acc[1], t[0], t[1])
        assert np.array_equal(acc[0], whole[0]) and np.array_equal(acc[1], whole[1])


def test_powerlaw_stream_is_sliceable_and_heavy_tailed(oracle):
    """The power-law generator (sheep_amd/csrc/powerlaw.h, host side): slices concatenate to
    the stream, ids stay in [0, n), and the degree distribution has a hub head and a long tail."""
    n, m = 50000, 400000
    uv = oracle.powerlaw(n, m, 2.3, 100.0, 3)
    assert uv.shape == (m, 2) and uv.max() < n
    assert np.array_equal(np.concatenate([oracle.powerlaw(n, m, 2.3, 100.0, 3, 0, 1234),
                                          oracle.powerlaw(n, m, 2.3, 100.0, 3, 1234, m)]), uv)
    deg = np.bincount(uv.ravel(), minlength=n)
    assert deg.max() > 30 * deg.mean()          # hubs
    assert np.median(deg) < 0.7 * deg.mean()    # most ids below the mean: a long tail


def test_ir_analogue_equals_serial_tree(oracle):
    """The `graph2tree -ir` CPU baseline (T shards, per-shard trees, log2(T) merge reduce) builds
    the serial tree (its own check flag), for T not a power of two too."""
    uv = oracle.rmat(12, 16, 9)
    for T in (1, 3, 4):
        _, _, _, n, ok = oracle.time_graph2tree_ir(uv, 1 << 12, T)
        assert ok and n == len(oracle.degree_sequence(uv))
