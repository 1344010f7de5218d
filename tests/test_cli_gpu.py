"""The four CLIs end to end on the GPU, against the CPU checker and the published hep-th run."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
PUB = json.load(open(os.path.join(GOLDEN, "hep_th_published.json")))
BIN = os.path.join(ROOT, "sheep_amd", "bin")
HEP = os.path.join(GOLDEN, "hep-th.dat")


def run(*args):
    return subprocess.run([os.path.join(BIN, args[0])] + list(args[1:]), capture_output=True,
                          text=True, check=True).stdout


def read_tre(path):
    raw = np.fromfile(path, dtype=np.uint32)
    body = raw[1:].reshape(-1, 2)[: int(raw[0])]
    return body[:, 0].copy(), body[:, 1].copy()


def test_graph2tree_faqs_and_timers(gpu, tmp_path):
    out = run("graph2tree", HEP, "-f", "-c")
    for line in ("Loaded graph in:", "Sorted in:", "Mapped in:", "Tree is valid."):
        assert line in out
    f = PUB["treefaqs"]
    assert "TREEFAQS: width:%d\troots:%d" % (f["width"], f["roots"]) in out
    assert "verts:%d\tedges:%d" % (f["verts"], f["edges"]) in out
    assert "halo:%d\tcore:%d" % (f["halo"], f["core"]) in out


def test_graph2tree_tre_equals_checker(gpu, oracle, hep_edges, tmp_path):
    tre = str(tmp_path / "hep.tre")
    run("graph2tree", HEP, "-o", tre)
    assert os.path.getsize(tre) == 60884
    p, s = read_tre(tre)
    op, os_ = oracle.build_tree(hep_edges, oracle.degree_sequence(hep_edges))
    assert np.array_equal(p, op) and np.array_equal(s, os_)


def test_partition_tree_degree_sequence_from_gpu(gpu, tmp_path):
    """partition_tree -g G - T k: the '-' sequence is degreeSequence on the GPU."""
    tre = str(tmp_path / "hep.tre")
    run("graph2tree", HEP, "-o", tre)
    out = run("partition_tree", "-f", "-g", HEP, "-", tre, "2", "16", "32")
    downs = [int(x) for x in re.findall(r"ECV\(down\): (\d+)", out)]
    want = {r["k"]: r["ecv_down"] for r in PUB["partitions"]}
    assert downs == [want[2], want[16], want[32]]


def test_degree_sequence_file_mode(gpu, oracle, tmp_path):
    sq = str(tmp_path / "hep.fseq")
    out = run("degree_sequence", HEP, sq)
    assert out.startswith("Sorted in: ")
    got = np.array([int(x) for x in open(sq).read().split()], np.uint32)
    assert np.array_equal(got, oracle.degree_sequence(oracle.read_dat_xs1reader(HEP), oracle.FILE))


def test_partial_loads_and_merge_trees(gpu, oracle, hep_edges, tmp_path):
    """graph2tree -l i/k -s SEQ partial trees, pairwise merge_trees == the serial tree
    (README:112-121; scripts/map-worker.sh + reduce-worker.sh)."""
    sq = str(tmp_path / "hep.seq")
    seq = oracle.degree_sequence(hep_edges)
    open(sq, "w").write("".join("%d\n" % x for x in seq))
    k = 4
    parts = []
    for i in range(1, k + 1):
        t = str(tmp_path / ("P%d.tre" % i))
        run("graph2tree", HEP, "-l", "%d/%d" % (i, k), "-s", sq, "-o", t)
        parts.append(t)
    run("merge_trees", parts[0], parts[1], "-o", str(tmp_path / "A.tre"))
    run("merge_trees", parts[2], parts[3], "-o", str(tmp_path / "B.tre"))
    out = run("merge_trees", "-f", str(tmp_path / "A.tre"), str(tmp_path / "B.tre"), "-o",
              str(tmp_path / "M.tre"))
    p, s = read_tre(str(tmp_path / "M.tre"))
    op, os_ = oracle.build_tree(hep_edges, seq)
    assert np.array_equal(p, op) and np.array_equal(s, os_)
    assert "halo:%d" % PUB["treefaqs"]["halo"] in out


def test_graph2tree_partition_output(gpu, oracle, hep_edges, tmp_path):
    """graph2tree -p K -o PREFIX: the fast partition path (graph2tree.cpp:203-216)."""
    prefix = str(tmp_path / "hp")
    run("graph2tree", HEP, "-p", "4", "-o", prefix)
    seq = oracle.degree_sequence(hep_edges)
    p, s = oracle.build_tree(hep_edges, seq)
    parts = oracle.PartTree(p, s).partition(seq, 4)
    # writePartitionedGraph (partition.cpp:588-630): every record (X, Y), X < Y once (self-loops
    # skipped), to the part of its lower-sequence endpoint; compared as per-file multisets
    # (the line order follows LLAMA's adjacency order, which no reference fixture pins)
    pos = np.full(parts.size, -1, np.int64)
    pos[seq] = np.arange(seq.size)
    x = hep_edges.min(axis=1).astype(np.int64)
    y = hep_edges.max(axis=1).astype(np.int64)
    keep = x != y
    x, y = x[keep], y[keep]
    owner = np.where(pos[x] < pos[y], parts[x], parts[y])
    created = int(parts.max()) + 1
    for q in range(created):
        lines = sorted(tuple(int(v) for v in l.split()) for l in open("%s%04d" % (prefix, q)))
        want = sorted(zip(x[owner == q].tolist(), y[owner == q].tolist()))
        assert lines == want, q
    assert not os.path.exists("%s%04d" % (prefix, created))


def test_partition_tree_gpu_evaluation_prints_the_same(gpu, tmp_path):
    """partition_tree -G evaluates on the GPU (sheep_evaluate): every evaluation line equals the
    host evaluation's, and ECV(down) the published one, for k = 2, 16, 32."""
    tre = str(tmp_path / "hep.tre")
    run("graph2tree", HEP, "-o", tre)
    host = run("partition_tree", "-g", HEP, "-", tre, "2", "16", "32")
    dev = run("partition_tree", "-G", "-g", HEP, "-", tre, "2", "16", "32")
    keep = re.compile(r"^(edges cut|Vcom|ECV|  balance)")
    h = [l for l in host.splitlines() if keep.match(l)]
    d = [l for l in dev.splitlines() if keep.match(l)]
    assert len(h) == 3 * 9 and d == h
    want = {r["k"]: r["ecv_down"] for r in PUB["partitions"]}
    assert [int(x) for x in re.findall(r"ECV\(down\): (\d+)", dev)] == [want[2], want[16], want[32]]


@pytest.mark.parametrize("flags", [["-i", "-r"], ["-r"]])
def test_graph2tree_mpi_flags_one_rank(gpu, oracle, hep_edges, tmp_path, flags):
    """graph2tree -i -r (mpiSequence + the collective tree) and -r -s SEQ (partial tree +
    mpi_merge) as one rank of an RCCL group (graph2tree.cpp:134-201): the saved tree equals the
    checker's, the seq file the checker's sequence, and the reduce timer line is printed."""
    tre = str(tmp_path / "m.tre")
    sq = str(tmp_path / "m.seq")
    seq = oracle.degree_sequence(hep_edges)
    if "-i" not in flags:
        open(sq, "w").write("".join("%d\n" % x for x in seq))
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               SHEEP_COMM_DIR=str(tmp_path), SHEEP_COMM_KEY="t")
    out = subprocess.run([os.path.join(BIN, "graph2tree"), HEP] + flags + ["-s", sq, "-o", tre],
                         capture_output=True, text=True, check=True, env=env).stdout
    assert "Reduced in:" in out
    p, s = read_tre(tre)
    op, os_ = oracle.build_tree(hep_edges, seq)
    assert np.array_equal(p, op) and np.array_equal(s, os_)
    got = np.array([int(x) for x in open(sq).read().split()], np.uint32)
    assert np.array_equal(got, seq)
