"""partition_tree (host C++ CLI, sheep_amd/bin) against the reference's published hep-th run.

The tree and the sequence come from the CPU checker, so this runs without a GPU: with a
sequence file, partition_tree's -g path (Partition + evaluate) is host code only.  The
published log (data/quality/hep.degree.raw) was one partition_tree run over k = 2..32.
"""
import json
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

PUB = json.load(open(os.path.join(GOLDEN, "hep_th_published.json")))
BIN = os.path.join(ROOT, "sheep_amd", "bin")


@pytest.fixture(scope="module")
def tools():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "sheep_amd", "tools")], check=True)
    return BIN


def write_tre(path, parent, pst):
    body = np.empty((len(parent), 2), np.uint32)
    body[:, 0], body[:, 1] = parent, pst
    with open(path, "wb") as f:
        f.write(np.uint32(len(parent)).tobytes())
        f.write(body.tobytes())


def parse_blocks(text):
    blocks = text.split("Partitioning took:")[1:]
    out = []
    for b in blocks:
        rec = {}
        m = re.search(r"Actually created (\d+) partitions", b)
        rec["created"] = int(m.group(1))
        m = re.search(r"First two partition sizes: (\d+) and (\d+)", b)
        rec["size0"], rec["size1"] = int(m.group(1)), int(m.group(2))
        for key, label in (("edges_cut", "edges cut"), ("vcom_vol", r"Vcom\. vol"),
                           ("ecv_hash", r"ECV\(hash\)"), ("ecv_down", r"ECV\(down\)"),
                           ("ecv_up", r"ECV\(up\)\s*")):
            mm = re.search(label + r": (\d+) \(([0-9.]+)%\)", b)
            rec[key], rec[key + "_pct"] = int(mm.group(1)), mm.group(2)
        out.append(rec)
    return out


def test_partition_tree_matches_published_hep_th(oracle, hep_edges, tools, tmp_path):
    seq = oracle.degree_sequence(hep_edges)
    p, s = oracle.build_tree(hep_edges, seq)
    tre, sq = str(tmp_path / "hep.tre"), str(tmp_path / "hep.seq")
    write_tre(tre, p, s)
    open(sq, "w").write("".join("%d\n" % x for x in seq))
    ks = [str(r["k"]) for r in PUB["partitions"]]
    out = subprocess.run([os.path.join(tools, "partition_tree"), "-f", "-g",
                          os.path.join(GOLDEN, "hep-th.dat"), sq, tre] + ks,
                         capture_output=True, text=True, check=True).stdout
    f = PUB["treefaqs"]
    assert "TREEFAQS: width:%d\troots:%d\n" % (f["width"], f["roots"]) in out
    assert "\tvheight:%d\teheight:%d\n" % (f["vheight"], f["eheight"]) in out
    assert "\thalo:%d\tcore:%d\n" % (f["halo"], f["core"]) in out
    got = parse_blocks(out)
    assert len(got) == len(PUB["partitions"])
    for g, want in zip(got, PUB["partitions"]):
        for key, val in g.items():
            assert val == want[key], (want["k"], key)


def test_partition_tree_balance_matches_checker(oracle, hep_edges, tools, tmp_path):
    """The balance lines (not in the published log) against the CPU checker, k = 2, 16."""
    seq = oracle.degree_sequence(hep_edges)
    p, s = oracle.build_tree(hep_edges, seq)
    tre, sq = str(tmp_path / "hep.tre"), str(tmp_path / "hep.seq")
    write_tre(tre, p, s)
    open(sq, "w").write("".join("%d\n" % x for x in seq))
    out = subprocess.run([os.path.join(tools, "partition_tree"), "-g",
                          os.path.join(GOLDEN, "hep-th.dat"), sq, tre, "2", "16"],
                         capture_output=True, text=True, check=True).stdout
    bal = [int(x) for x in re.findall(r"balance: (\d+) \(", out)]
    pt = oracle.PartTree(p, s)
    want = []
    for k in (2, 16):
        ev = oracle.evaluate(hep_edges, pt.partition(seq, k), seq)
        want += [ev["vertex_bal"], ev["hash_bal"], ev["down_bal"], ev["up_bal"]]
    assert bal == want
    assert re.findall(r"ECV\(down\): (\d+)", out) == ["521", "2425"]  # SURVEY §8c probe


def test_partition_tree_writes_partitioned_edges(oracle, hep_edges, tools, tmp_path):
    """-g G -o OUT: every record goes to the part of its lower-sequence endpoint."""
    seq = oracle.degree_sequence(hep_edges)
    p, s = oracle.build_tree(hep_edges, seq)
    tre, sq = str(tmp_path / "hep.tre"), str(tmp_path / "hep.seq")
    write_tre(tre, p, s)
    open(sq, "w").write("".join("%d\n" % x for x in seq))
    prefix = str(tmp_path / "part")
    subprocess.run([os.path.join(tools, "partition_tree"), "-g", os.path.join(GOLDEN, "hep-th.dat"),
                    "-o", prefix, sq, tre, "4"], capture_output=True, text=True, check=True)
    parts = oracle.PartTree(p, s).partition(seq, 4)
    pos = np.full(int(seq.max()) + 1, -1)
    pos[seq] = np.arange(len(seq))
    stream = oracle.read_dat_xs1reader(os.path.join(GOLDEN, "hep-th.dat"))
    want = {}
    for x, y in stream:
        q = parts[x] if pos[x] < pos[y] else parts[y]
        want.setdefault(int(q), []).append((int(x), int(y)))
    for q, edges in want.items():
        got = [tuple(map(int, l.split())) for l in open("%s%04d" % (prefix, q))]
        assert got == edges
