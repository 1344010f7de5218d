"""GPU parity: libsheep_amd.so (HIP, gfx950) against the CPU checker, bit-exact.

Inputs: the reference's hep-th fixture, the known-answer graph, seeded R-MAT streams (the GPU
generator is itself checked against the host generator), random multigraphs with self-loops
and duplicates, and the edge cases the reference defines (empty input, isolated ids, repeated
seq ids, ids outside the sequence).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
PUB = json.load(open(os.path.join(GOLDEN, "hep_th_published.json")))
KA = json.load(open(os.path.join(GOLDEN, "known_answer.json")))


@pytest.fixture(scope="module")
def api(gpu):
    from sheep_amd import api

    return api


def check_tree(O, api, uv, seq):
    t = api.build_tree(uv, seq)
    p, s = O.build_tree(uv, seq)
    assert np.array_equal(t.parent, p), "parent mismatch"
    assert np.array_equal(t.pst, s), "pst mismatch"
    return t


def test_known_answer(oracle, api):
    uv = np.array(KA["records"], np.uint32)
    seq = api.degree_sequence(uv)
    assert seq.tolist() == KA["llama_seq"]
    t = api.build_tree(uv, seq)
    assert [-1 if x == 0xFFFFFFFF else int(x) for x in t.parent] == KA["parent"]
    assert t.pst.tolist() == KA["pst"]
    assert api.degree_sequence(uv, api.DEGREE_FILE).tolist() == KA["file_seq_stream"]


def test_hep_th_llama(oracle, api, hep_edges):
    seq = api.degree_sequence(hep_edges)
    assert np.array_equal(seq, oracle.degree_sequence(hep_edges))
    t = check_tree(oracle, api, hep_edges, seq)
    assert oracle.facts(t.parent, t.pst) == PUB["treefaqs"]


def test_hep_th_file_mode_and_reader(oracle, api):
    path = os.path.join(GOLDEN, "hep-th.dat")
    fseq = api.file_sequence(path)
    assert np.array_equal(fseq, oracle.degree_sequence(oracle.read_dat_xs1reader(path), oracle.FILE))
    uv = api.read_dat(path)
    t = check_tree(oracle, api, uv, fseq)
    assert oracle.facts(t.parent, t.pst)["halo"] == 3530  # SURVEY A2 probe: FILE-mode seq


@pytest.mark.parametrize("scale,seed", [(10, 1), (12, 2), (14, 3), (16, 4)])
def test_rmat_generator_and_tree(oracle, api, gpu, scale, seed):
    import torch
    from sheep_amd import device

    uv_d = device.rmat(scale, 16, seed)
    uv = uv_d.cpu().numpy().view(np.uint32)
    assert np.array_equal(uv, oracle.rmat(scale, 16, seed))
    seq = api.degree_sequence(uv)
    assert np.array_equal(seq, oracle.degree_sequence(uv))
    check_tree(oracle, api, uv, seq)
    # fused device pipeline
    s_d, p_d, w_d, n = device.graph2tree(uv_d, 1 << scale)
    torch.cuda.synchronize()
    p, w = oracle.build_tree(uv, seq)
    assert n == len(seq)
    assert np.array_equal(s_d[:n].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:n].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:n].cpu().numpy().view(np.uint32), w)


def _degrees(case, rng):
    if case == "heavy":     # zipf tail: every counting class, hundreds of ids above 1024
        d = np.minimum(rng.zipf(1.6, 300001), 1 << 31).astype(np.uint32)
        d[rng.random(d.size) < 0.3] = 0
    elif case == "small":   # no id reaches the radix-sorted class
        d = rng.integers(0, 50, 5000, dtype=np.uint32)
    elif case == "ones":    # one class, off the 16384-id chunk
        d = np.ones(40000, np.uint32)
        d[rng.integers(0, d.size, 100)] = 0
    elif case == "zeros":
        d = np.zeros(20000, np.uint32)
    elif case == "full":    # degrees over the whole u32 range, and the class edges 1023/1024
        d = rng.integers(0, 1 << 32, 70000, dtype=np.uint64).astype(np.uint32)
        m = rng.random(d.size) < 0.5
        d[m] = rng.integers(1020, 1028, int(m.sum()), dtype=np.uint32)
        d[::7] = 1023
        d[::11] = 1024
        d[-1] = 0xFFFFFFFF
    else:                   # one id
        d = np.array([5], np.uint32)
    return d


@pytest.mark.parametrize("case", ["heavy", "small", "ones", "zeros", "full", "one"])
def test_sequence_from_degrees(oracle, gpu, case):
    """sheep_sequence_dev on crafted degree vectors (sequence.h:55-61: degree > 0, by degree,
    ties in id order): the counting sort's classes below 1024 and the radix-sorted ids above,
    ties, zero degrees, sizes off its 16384-id chunk, degrees up to 2^32-1."""
    import torch
    from sheep_amd import device

    d = _degrees(case, np.random.default_rng(len(case)))
    seq, rank, n = device.sequence(torch.from_numpy(d.view(np.int32)).cuda().view(torch.uint32))
    torch.cuda.synchronize()
    want = oracle.sequence(d)
    assert n == want.size
    assert np.array_equal(seq[:n].cpu().numpy().view(np.uint32), want)
    rk = np.full(d.size, 0xFFFFFFFF, np.uint32)
    rk[want] = np.arange(want.size, dtype=np.uint32)
    assert np.array_equal(rank[:d.size].cpu().numpy().view(np.uint32), rk)


@pytest.mark.parametrize("scale,seed,mode,env", [
    (18, 21, 0, {}),                        # partitioned gathers (m >= 2^22), overlapped pass 1
    (18, 22, 1, {}),                        # FILE degrees: self-loops count twice in pst's degree
    (16, 23, 0, {"edge_part": 1}),  # the partitioned gathers at a small size
    (18, 24, 0, {"bin_slack": -900}),       # direct bins at 1/10 of the estimate: they overflow
                                            # and the records are grouped again by the scatter
    (16, 25, 0, {"bin_slack": -900, "edge_part": 0}),  # the same from unpartitioned records
    (17, 26, 0, {"bin_direct": 0}),         # edge pass + bin scatter (no direct binning)
    (16, 24, 0, {"edge_part": 0}),  # direct gathers, hi bins
    (18, 26, 1, {"kb_pipe": 0}),    # one stream: rebase, map, apply in turn
    (18, 29, 0, {"bin_direct": 0}),                    # edge pass + bin scatter
    (18, 30, 0, {"part_overlap": 3}),  # fused: the degree scatter partitions the records
    (18, 32, 1, {"part_overlap": 3}),  # fused, FILE degrees
    (18, 31, 1, {"part_overlap": 0}),  # the first partition pass in line
    (18, 33, 0, {"kb_rlink": 0}),   # every kept pair through the zipper's lane queue
    (18, 34, 1, {"kb_rlink": 0, "kb_pipe": 0}),
])
def test_graph2tree_dev_front_half(oracle, gpu, options, scale, seed, mode, env):
    """The fused device pipeline (sheep_graph2tree_dev) where the rank gathers are partitioned
    and the first partition pass runs beside the degree pass and the sequence sort, with the
    compacted sequence sort, tile-major bin counts and the unstable bin scatter: seq, parent
    and pst bit-exact against the checker in both degree conventions."""
    import torch
    from sheep_amd import device

    options(**env)
    uv_d = device.rmat(scale, 16, seed)
    uv = uv_d.cpu().numpy().view(np.uint32)
    seq = oracle.degree_sequence(uv, mode)
    s_d, p_d, w_d, n = device.graph2tree(uv_d, 1 << scale, mode)
    torch.cuda.synchronize()
    p, w = oracle.build_tree(uv, seq)
    assert n == len(seq)
    assert np.array_equal(s_d[:n].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:n].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:n].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("mode,ov,ff", [(0, 4, 8), (1, 4, 8), (0, 4, 1), (1, 4, 3), (0, 2, 8),
                                        (1, 2, 8)])
def test_graph2tree_dev_sampled_capacities(oracle, gpu, options, mode, ov, ff):
    """From 2^25 records the front half writes into capacity regions sized from a 1/256 sample
    of the records (no counting read): one fused read for the degrees and the packed first
    partition (part_overlap 4, k_front_fused; ff tile groups, each with its own subregion of
    every region, read back through the second pass's tile map), or the degree scatter beside
    the first partition pass (2).  R-MAT 21 (2^25 records), seq / parent / pst bit-exact in
    both degree conventions, the exact pass not needed."""
    import torch
    from sheep_amd import capi, device

    options(part_overlap=ov, ff_groups=ff)
    uv_d = device.rmat(21, 16, 77 + mode)
    s_d, p_d, w_d, n = device.graph2tree(uv_d, 1 << 21, mode)
    torch.cuda.synchronize()
    t = dict(capi.last_timings())
    assert "degree_exact" not in t
    assert ("front_fused" in t) == (ov == 4)
    uv = uv_d.cpu().numpy().view(np.uint32)
    seq = oracle.degree_sequence(uv, mode)
    p, w = oracle.build_tree(uv, seq)
    assert n == len(seq)
    assert np.array_equal(s_d[:n].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:n].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:n].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("ff", [8, 1])
def test_graph2tree_dev_fused_groups_sorted_stream(oracle, gpu, options, ff):
    """The fused pass's tile groups on a stream sorted by tail (an adjacency-ordered file): each
    group's records of a region then come from a few tiles, so the subregions' sizes follow the
    order, not the shares of a shuffled stream.  The per-group sample sees the same order;
    whatever it misjudges goes through the overflow paths.  R-MAT 21 sorted by (tail, head),
    bit-exact."""
    import torch
    from sheep_amd import device

    options(ff_groups=ff)
    uv = device.rmat(21, 16, 91).cpu().numpy().view(np.uint32)
    uv = uv[np.lexsort((uv[:, 1], uv[:, 0]))]
    uv_d = torch.from_numpy(np.ascontiguousarray(uv).view(np.int32)).cuda().view(torch.uint32)
    s_d, p_d, w_d, n = device.graph2tree(uv_d, 1 << 21)
    torch.cuda.synchronize()
    seq = oracle.degree_sequence(uv)
    p, w = oracle.build_tree(uv, seq)
    assert n == len(seq)
    assert np.array_equal(s_d[:n].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:n].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:n].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("ov", [4, 2])
def test_graph2tree_dev_sampled_capacities_overflow(oracle, gpu, options, ov):
    """An input the sample misjudges: every 256th record (the sampled ones) joins ids 0 and 1,
    the others spread over 2^20 ids, so every other degree bucket and y digit outgrows its
    capacity.  The degrees go through the exact pass (and the partition through the hi bins'
    fallback): still bit-exact, fused (4) or not (2)."""
    import torch
    from sheep_amd import capi, device

    options(part_overlap=ov)
    m, n_ids = 1 << 25, 1 << 20
    rng = np.random.default_rng(3)
    uv = rng.integers(0, n_ids, size=(m, 2), dtype=np.uint32)
    uv[::256] = (0, 1)
    uv_d = torch.from_numpy(uv.view(np.int32)).cuda().view(torch.uint32)
    s_d, p_d, w_d, n = device.graph2tree(uv_d, n_ids)
    torch.cuda.synchronize()
    assert "degree_exact" in dict(capi.last_timings())
    seq = oracle.degree_sequence(uv)
    p, w = oracle.build_tree(uv, seq)
    assert n == len(seq)
    assert np.array_equal(s_d[:n].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:n].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:n].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("ff", [8, 1])
def test_graph2tree_dev_fused_y_overflow_only(oracle, gpu, options, ff):
    """Only the y regions overflow: every 256th record (the sampled ones) has a uniform head, the
    others a head in one y digit's 1024 ids, while the tails stay uniform (the x buckets fit).
    The fused pass's histogram counts the heads from the packed records, so a dropped y run
    loses degrees too: the exact degree pass must run on the y flag alone (round 6; it ran on the
    x flag only).  Bit-exact."""
    import torch
    from sheep_amd import capi, device

    options(ff_groups=ff)
    m, n_ids = 1 << 25, 1 << 20
    rng = np.random.default_rng(21)
    uv = rng.integers(0, n_ids, size=(m, 2), dtype=np.uint32)
    keep = np.zeros(m, bool)
    keep[::256] = True
    uv[~keep, 1] = rng.integers(5 << 10, 6 << 10, size=int((~keep).sum()), dtype=np.uint32)
    uv_d = torch.from_numpy(uv.view(np.int32)).cuda().view(torch.uint32)
    s_d, p_d, w_d, n = device.graph2tree(uv_d, n_ids)
    torch.cuda.synchronize()
    assert "degree_exact" in dict(capi.last_timings())
    seq = oracle.degree_sequence(uv)
    p, w = oracle.build_tree(uv, seq)
    assert n == len(seq)
    assert np.array_equal(s_d[:n].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:n].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:n].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("ov", [4, 2])
def test_graph2tree_dev_sampled_overflow_few_ids(oracle, gpu, options, ov):
    """The sampled regions overflow on an input with at most 256 ids in use: the
    tree then takes no hi bins (n_seq <= 256), so the direct edge pass, which used to be the
    only reader of the first pass's overflow word, does not run.  Every 256th record (the
    sampled ones) joins ids 0 and 1, the others join 200 ids spread over 2^20 (one per y digit,
    none of which the sample saw).  Bit-exact, fused (4) or not (2)."""
    import torch
    from sheep_amd import device

    options(part_overlap=ov)
    m, n_ids = 1 << 25, 1 << 20
    rng = np.random.default_rng(4)
    ids = (np.arange(1, 201, dtype=np.uint32) * 5003) % n_ids
    uv = ids[rng.integers(0, ids.size, size=(m, 2))]
    uv[::256] = (0, 1)
    uv_d = torch.from_numpy(uv.view(np.int32)).cuda().view(torch.uint32)
    s_d, p_d, w_d, n = device.graph2tree(uv_d, n_ids)
    torch.cuda.synchronize()
    seq = oracle.degree_sequence(uv)
    p, w = oracle.build_tree(uv, seq)
    assert n == len(seq) <= 256
    assert np.array_equal(s_d[:n].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:n].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:n].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("n,m,mode", [((1 << 26) + 5, (1 << 22) + 12345, 0),
                                      ((1 << 25) + 77, (1 << 22) + 1, 1)])
def test_graph2tree_dev_fused_64k_buckets(oracle, gpu, options, n, m, mode):
    """The fused front half (launch_fh_front) with 64K-id buckets (n_ids > 2^25: the one-read
    u16 histogram over the records' y ids then the x ids) and a ragged last chunk: seq, parent
    and pst bit-exact in both degree conventions."""
    import torch
    from sheep_amd import device

    options(part_overlap=3)

    uv_d = device.powerlaw(n, m, 2.2, 80.0, 9 + mode)
    uv = uv_d.cpu().numpy().view(np.uint32).reshape(-1, 2)
    seq = oracle.degree_sequence(uv, mode)
    s_d, p_d, w_d, k = device.graph2tree(uv_d, n, mode)
    torch.cuda.synchronize()
    p, w = oracle.build_tree(uv, seq)
    assert k == len(seq)
    assert np.array_equal(s_d[:k].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:k].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:k].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("mode", [0, 1])
def test_graph2tree_dev_fused_hub_fills_rounds(oracle, gpu, mode):
    """The fused pass's histogram counts a bucket in rounds of 65528 entries into u16 halves:
    a hub that is the ONLY id of its 64K-id bucket (35 % of 2^25 + 12345 records) fills every
    round of that bucket's endpoint region with itself, 65528 counts a round — one short of
    wrapping a half. Its degree (~11.7 M) and the tree must match the checker."""
    import torch
    from sheep_amd import capi, device

    rng = np.random.default_rng(11 + mode)
    n = (1 << 26) - 5
    m = (1 << 25) + 12345
    uv = rng.integers(0, n, size=(m, 2)).astype(np.uint32)
    hb = 5  # no other id of bucket 5 occurs
    for c in (0, 1):
        inb = (uv[:, c] >> 16) == hb
        uv[inb, c] += 1 << 16
    hub = (hb << 16) + 9
    sel = rng.random(m) < 0.35
    uv[sel, 0] = hub
    uv_d = torch.from_numpy(uv.view(np.int32)).cuda().view(torch.uint32)
    s_d, p_d, w_d, k = device.graph2tree(uv_d, n, mode)
    torch.cuda.synchronize()
    assert "front_fused" in dict(capi.last_timings())
    seq = oracle.degree_sequence(uv, mode)
    p, w = oracle.build_tree(uv, seq)
    assert k == len(seq) and seq[-1] == hub
    assert np.array_equal(s_d[:k].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:k].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:k].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("n,mode", [(3000017, 0), (40000003, 1)])
def test_graph2tree_dev_fused_ragged_ids(oracle, gpu, n, mode):
    """The default front half (the fused pass, sampled capacities) on id spaces that are not a
    power of two: 733 degree buckets of 4K ids (n = 3,000,017) or 611 of 64K ids (n =
    40,000,003), each with a ragged last bucket and y digit, over 2^25 + 999 power-law records
    (a ragged last tile): seq, parent and pst bit-exact in both degree conventions."""
    import torch
    from sheep_amd import capi, device

    m = (1 << 25) + 999
    uv_d = device.powerlaw(n, m, 2.2, 80.0, 40 + mode)
    s_d, p_d, w_d, k = device.graph2tree(uv_d, n, mode)
    torch.cuda.synchronize()
    assert "front_fused" in dict(capi.last_timings())
    uv = uv_d.cpu().numpy().view(np.uint32).reshape(-1, 2)
    seq = oracle.degree_sequence(uv, mode)
    p, w = oracle.build_tree(uv, seq)
    assert k == len(seq)
    assert np.array_equal(s_d[:k].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:k].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:k].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("n,m,gamma,i0,seed", [(1000, 20000, 2.3, 100.0, 3),
                                               (65536, 1 << 20, 2.1, 50.0, 5),
                                               (300001, 1 << 21, 2.3, 100.0, 7)])
def test_powerlaw_generator_and_tree(oracle, api, gpu, n, m, gamma, i0, seed):
    """The LJ/twitter-shape generator: the GPU stream equals the host stream (any slice), and
    the tree of a power-law graph (hubs, isolated ids, self-loops) is bit-exact."""
    import torch
    from sheep_amd import device

    uv_d = device.powerlaw(n, m, gamma, i0, seed)
    uv = uv_d.cpu().numpy().view(np.uint32)
    assert np.array_equal(uv, oracle.powerlaw(n, m, gamma, i0, seed))
    part = device.powerlaw(n, m, gamma, i0, seed, m // 3, m // 2).cpu().numpy().view(np.uint32)
    assert np.array_equal(part, uv[m // 3: m // 2])
    assert uv.max() < n
    s_d, p_d, w_d, k = device.graph2tree(uv_d, n)
    torch.cuda.synchronize()
    seq = oracle.degree_sequence(uv)
    p, w = oracle.build_tree(uv, seq)
    assert k == len(seq)
    assert np.array_equal(s_d[:k].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:k].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:k].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("seed", range(6))
def test_random_multigraphs(oracle, api, seed):
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(2, 3000))
    m = int(rng.integers(1, 20000))
    uv = rng.integers(0, n, size=(m, 2)).astype(np.uint32)
    dup = rng.integers(0, m, size=m // 10)
    uv = np.concatenate([uv, uv[dup]])  # duplicate records (a multigraph, no DDUP_GRAPH)
    loops = rng.random(len(uv)) < 0.03
    uv[loops, 1] = uv[loops, 0]
    for mode in (0, 1):
        seq = api.degree_sequence(uv, mode)
        assert np.array_equal(seq, oracle.degree_sequence(uv, mode))
        check_tree(oracle, api, uv, seq)


def test_random_seq_order(oracle, api):
    """Any total order works (readSequence path, graph2tree.cpp:171-174)."""
    uv = oracle.rmat(12, 8, 9)
    seq = oracle.degree_sequence(uv)
    rng = np.random.default_rng(5)
    check_tree(oracle, api, uv, rng.permutation(seq).astype(np.uint32))


def test_seq_subset_and_padding(oracle, api):
    """Ids missing from seq behave as INVALID index (POSTORDER for their neighbours); seq may
    carry ids with no edges (make_pad, jtree.h:88)."""
    uv = np.array([[0, 1], [1, 2], [2, 3], [3, 0], [1, 3]], np.uint32)
    seq = np.array([3, 1, 0, 7], np.uint32)  # 2 missing, 7 isolated
    check_tree(oracle, api, uv, seq)


def test_duplicate_seq_is_einval(api):
    uv = np.array([[0, 1]], np.uint32)
    with pytest.raises(api.SheepError) as e:
        api.build_tree(uv, np.array([0, 1, 0], np.uint32))
    assert e.value.code == -22


def test_neighbour_beyond_seq_is_erange(api):
    uv = np.array([[0, 1], [1, 5]], np.uint32)
    with pytest.raises(api.SheepError) as e:
        api.build_tree(uv, np.array([0, 1], np.uint32))
    assert e.value.code == -34


def test_corrupt_forest_trips_walk_guard(oracle, api):
    """A tree that is not heap-ordered (parent[1] = 0 < 1) would send the zipper's walk in a
    circle; the walk guard stops it and the call fails with -EIO (fault_word), after which the
    device works normally again (the guard word is cleared)."""
    inv = 0xFFFFFFFF
    a = api.JNodeTable(np.array([2, 0, inv], np.uint32), np.zeros(3, np.uint32))
    b = api.JNodeTable(np.array([1, inv, inv], np.uint32), np.zeros(3, np.uint32))
    with pytest.raises(api.SheepError) as e:
        api.merge_trees(a, b)
    assert e.value.code == -5
    good = api.JNodeTable(np.array([2, 2, inv], np.uint32), np.zeros(3, np.uint32))
    g = api.merge_trees(good, b)
    p, s = oracle.merge(good.parent, good.pst, b.parent, b.pst)
    assert np.array_equal(g.parent, p) and np.array_equal(g.pst, s)


def test_empty_and_isolated(oracle, api):
    assert api.degree_sequence(np.zeros((0, 2), np.uint32)).size == 0
    uv = np.array([[5, 5]], np.uint32)  # only a self-loop: one vertex, no tree edge
    seq = api.degree_sequence(uv)
    assert seq.tolist() == [5]
    t = check_tree(oracle, api, uv, seq)
    assert t.parent.tolist() == [0xFFFFFFFF] and t.pst.tolist() == [0]


@pytest.mark.parametrize("k", [2, 3, 4, 8])
def test_merge_of_shards_equals_whole(oracle, api, k):
    uv = oracle.rmat(14, 16, 11)
    seq = oracle.degree_sequence(uv)
    whole = oracle.build_tree(uv, seq)
    R = len(uv)
    trees = [api.build_tree(uv[R * i // k: R * (i + 1) // k], seq) for i in range(k)]
    for i, t in enumerate(trees):  # each partial tree is itself exact
        p, s = oracle.build_tree(uv[R * i // k: R * (i + 1) // k], seq)
        assert np.array_equal(t.parent, p) and np.array_equal(t.pst, s)
    step = 1
    while step < k:  # pairwise log2 reduce, as scripts/reduce-worker.sh
        for i in range(0, k - step, 2 * step):
            a, b = trees[i], trees[i + step]
            g = api.merge_trees(a, b)
            p, s = oracle.merge(a.parent, a.pst, b.parent, b.pst)
            assert np.array_equal(g.parent, p) and np.array_equal(g.pst, s)
            trees[i] = g
        step *= 2
    assert np.array_equal(trees[0].parent, whole[0]) and np.array_equal(trees[0].pst, whole[1])


def test_tre_roundtrip(api, hep_edges, tmp_path):
    seq, t = api.graph2tree(hep_edges)
    path = str(tmp_path / "h.tre")
    t.save(path)
    assert os.path.getsize(path) == 4 + 8 * len(seq)  # 60,884 B for hep-th
    assert api.JNodeTable.load(path) == t


@pytest.mark.parametrize("path", ["atomic", "bucketed"])
@pytest.mark.parametrize("seed", range(3))
def test_degree_paths_agree(oracle, api, options, path, seed):
    """Both degree kernels (global atomics / LDS-bucketed) on multigraphs with self-loops,
    in both degree conventions, including tiny id spaces (one id per bucket)."""
    options(degree={"atomic": 1, "bucketed": 2}[path])
    rng = np.random.default_rng(200 + seed)
    n = [3, 5000, 70000][seed]
    m = [50, 300000, 600000][seed]
    uv = rng.integers(0, n, size=(m, 2)).astype(np.uint32)
    loops = rng.random(m) < 0.05
    uv[loops, 1] = uv[loops, 0]
    hub = rng.random(m) < 0.2  # a hub: one id repeated across many waves
    uv[hub, 0] = 1
    for mode in (0, 1):
        assert np.array_equal(api.degree_sequence(uv, mode), oracle.degree_sequence(uv, mode))


@pytest.mark.parametrize("seed", range(3))
def test_sharded_partial_trees_with_degree_pst(oracle, gpu, seed):
    """sheep_degree_ex_dev + sheep_build_tree_deg_dev on edge shards (the multi-GPU per-rank
    step) equal the checker's partial trees, and their merges equal the whole tree."""
    import torch
    from sheep_amd import device

    scale, P = 13, 3
    uv_all = device.rmat(scale, 16, 40 + seed)
    uv = uv_all.cpu().numpy().view(np.uint32)
    # add self-loops and an id-space gap so the self-loop and missing-id paths are exercised
    uv = np.concatenate([uv, np.array([[5, 5], [5, 5], [7, 7]], np.uint32)])
    uv_d = torch.from_numpy(uv.view(np.int32)).cuda().view(torch.uint32)
    n_ids = 1 << scale
    deg = torch.zeros(n_ids, dtype=torch.uint32, device="cuda")
    shards = []
    R = len(uv)
    for r in range(P):
        sh = uv_d[R * r // P: R * (r + 1) // P].contiguous()
        d, sc = device.degree_ex(sh, n_ids)
        deg = (deg.view(torch.int32) + d.view(torch.int32)).view(torch.uint32)
        shards.append((sh, d, sc))
    seq, rank, n_seq = device.sequence(deg)
    oseq = oracle.degree_sequence(uv)
    assert n_seq == len(oseq) and np.array_equal(seq[:n_seq].cpu().numpy().view(np.uint32), oseq)
    acc = None
    parts = []
    for r, (sh, d, sc) in enumerate(shards):
        p, s = device.build_tree_deg(sh, rank, seq, n_seq, d, sc)
        parts.append(p[:n_seq].clone())
        op, os_ = oracle.build_tree(uv[R * r // P: R * (r + 1) // P], oseq)
        assert np.array_equal(p[:n_seq].cpu().numpy().view(np.uint32), op)
        assert np.array_equal(s[:n_seq].cpu().numpy().view(np.uint32), os_)
        if acc is None:
            acc = (p, s)
        else:
            device.merge_into(acc[0], acc[1], p, s, n_seq)
    torch.cuda.synchronize()
    wp, ws = oracle.build_tree(uv, oseq)
    assert np.array_equal(acc[0][:n_seq].cpu().numpy().view(np.uint32), wp)
    assert np.array_equal(acc[1][:n_seq].cpu().numpy().view(np.uint32), ws)
    # the multi-GPU reduce: one P-way union build over the gathered parent arrays
    mp = device.merge_forests(torch.stack(parts), n_seq)
    torch.cuda.synchronize()
    assert np.array_equal(mp[:n_seq].cpu().numpy().view(np.uint32), wp)


@pytest.mark.parametrize("P", [1, 2, 5, 8])
def test_merge_forests_equals_whole(oracle, gpu, P):
    """sheep_merge_forests_dev over P partial trees (scale 14) is the whole graph's tree, and
    the union of a forest with itself or with an empty forest is that forest."""
    import torch
    from sheep_amd import device

    uv = oracle.rmat(14, 16, 90 + P)
    seq = oracle.degree_sequence(uv)
    n = len(seq)
    R = len(uv)
    parts = [oracle.build_tree(uv[R * r // P: R * (r + 1) // P], seq)[0] for r in range(P)]
    stack = torch.from_numpy(np.stack(parts).view(np.int32)).cuda().view(torch.uint32)
    got = device.merge_forests(stack, n)
    wp, _ = oracle.build_tree(uv, seq)
    assert np.array_equal(got[:n].cpu().numpy().view(np.uint32), wp)
    twice = device.merge_forests(torch.stack([got[:n], got[:n]]), n)
    empty = torch.full((n,), 0xFFFFFFFF, dtype=torch.int64).to(torch.int32).cuda().view(torch.uint32)
    with_empty = device.merge_forests(torch.stack([empty, got[:n]]), n)
    torch.cuda.synchronize()
    assert np.array_equal(twice[:n].cpu().numpy().view(np.uint32), wp)
    assert np.array_equal(with_empty[:n].cpu().numpy().view(np.uint32), wp)


KB_KNOBS = [
    {},                                              # defaults (giant bitmap + spine)
    {"kb_buckets": 4, "kb_rankb": 8},                # few, wide buckets
    {"kb_buckets": 512},                             # many buckets
    {"kb_pipe": 0},                                  # one stream, map of bucket k after apply of k-1
    {"kb_pipe": 1, "kb_buckets": 512, "kb_rankb": 512},  # many narrow buckets
    {"kb_gsum": 0},                                  # no LDS giant summary in the map
    {"kb_gsum": 1},                                  # the summary at every size (auto: 2^27 records)
]


@pytest.mark.parametrize("knobs", KB_KNOBS, ids=lambda k: ",".join("%s=%s" % kv for kv in k.items()) or "default")
@pytest.mark.parametrize("scale,seed", [(15, 5), (17, 6)])
def test_tree_knobs_exact(oracle, api, options, knobs, scale, seed):
    """The tree is the same unique etree under every bucketing / bitmap / queue setting: the
    knobs change the work, never the result (R-MAT, where a giant component forms)."""
    options(**knobs)
    uv = oracle.rmat(scale, 16, seed)
    seq = oracle.degree_sequence(uv)
    check_tree(oracle, api, uv, seq)
    rng = np.random.default_rng(seed)
    check_tree(oracle, api, uv, rng.permutation(seq).astype(np.uint32))  # no giant at the end


def _eval_case(oracle, uv, k, seed, random_parts=False):
    """Checker tree -> checker partition (forwardPartition; or random parts) -> GPU and
    checker evaluate."""
    import torch
    from sheep_amd import device

    seq = oracle.degree_sequence(uv)
    if random_parts:
        parts = np.random.default_rng(seed).integers(0, k, int(seq.max()) + 1).astype(np.int16)
    else:
        p, s = oracle.build_tree(uv, seq)
        parts = oracle.PartTree(p, s).partition(seq, k)
    n_ids = int(uv.max()) + 1
    parts_full = np.full(n_ids, -1, np.int16)
    parts_full[:parts.size] = parts
    uv_d = torch.from_numpy(np.ascontiguousarray(uv).view(np.int32)).cuda().view(torch.uint32)
    rank = np.full(n_ids, 0xFFFFFFFF, np.uint32)
    rank[seq] = np.arange(seq.size, dtype=np.uint32)
    rank_d = torch.from_numpy(rank.view(np.int32)).cuda().view(torch.uint32)
    parts_d = torch.from_numpy(parts_full).cuda()
    got = device.evaluate(uv_d, parts_d, rank_d, n_parts=int(parts.max()) + 1)
    want = oracle.evaluate(uv, parts, seq)
    return got, want


@pytest.mark.parametrize("k", [2, 16, 64])
def test_evaluate_hep_th_matches_checker_and_published(oracle, api, hep_edges, k):
    """Partition::evaluate on the GPU == the checker's, on hep-th (published ECV(down) for
    k = 2, 16 is pinned in test_oracle_golden)."""
    got, want = _eval_case(oracle, hep_edges, k, 0)
    assert got == want


@pytest.mark.parametrize("scale,k", [(12, 4), (14, 256), (16, 32)])
def test_evaluate_rmat_matches_checker(oracle, api, scale, k):
    """R-MAT streams carry self-loops and duplicate records: both adjacency conventions of the
    evaluation (a self-loop is one entry; duplicates count) are exercised."""
    uv = oracle.rmat(scale, 16, 70 + scale)
    got, want = _eval_case(oracle, uv, k, scale)
    assert got == want


@pytest.mark.parametrize("scale,k,ep", [(14, 16, 16), (16, 64, 18)])
def test_evaluate_in_id_range_passes(oracle, api, options, scale, k, ep):
    """The evaluation's id-range passes (taken beyond 2^31 adjacency entries, e.g. a 2^31-record
    graph), forced here at 2^ep entries per pass: every number equals the checker's."""
    options(eval_pass=ep)
    uv = oracle.rmat(scale, 16, 90 + scale)
    got, want = _eval_case(oracle, uv, k, scale)
    assert got == want


def test_evaluate_many_parts_global_histograms(oracle, api):
    """k above the LDS histogram limit (2048 parts) takes the global-atomics path (random
    parts: forwardPartition at this k is slow in the checker)."""
    uv = oracle.rmat(13, 16, 5)
    got, want = _eval_case(oracle, uv, 3000, 1, random_parts=True)
    assert got == want


def test_evaluate_rejects_missing_part(api):
    import torch
    from sheep_amd import capi, device

    uv = torch.tensor([[0, 1], [1, 2]], dtype=torch.int32).cuda().view(torch.uint32)
    parts = torch.tensor([0, -1, 0], dtype=torch.int16).cuda()
    rank = torch.tensor([0, 1, 2], dtype=torch.int32).cuda().view(torch.uint32)
    with pytest.raises(capi.SheepError) as e:
        device.evaluate(uv, parts, rank, n_parts=1)
    assert e.value.code == -34  # -ERANGE


def test_degree_64k_id_buckets_repeatable(api, options):
    """The 64K-id histogram on a skewed power law (41.6 M ids, 2^28 records, hub degrees in the
    hundreds of thousands): three passes give identical degrees summing to 2m - self-loops
    (LLAMA). Guards the LDS-draining barriers: with a barrier compiled without the wait, late
    LDS adds of one wave were lost or moved run to run."""
    import torch
    from sheep_amd import capi, device

    options(degree=2)
    n_ids, m = 41652230, 1 << 28
    uv = device.powerlaw(n_ids, m, 2.1, 50.0, 5, 0, m)
    u = uv.view(torch.int32)
    loops = int((u[:, 0] == u[:, 1]).sum())
    ref = None
    for _ in range(3):
        d = device.degree(uv, n_ids, capi.DEGREE_LLAMA).view(torch.int32).to(torch.int64)
        assert int(d.sum()) == 2 * m - loops
        if ref is None:
            ref = d
        else:
            assert torch.equal(d, ref)


def test_degree_64k_id_buckets(oracle, api, options):
    """Id spaces above 2^25 use buckets of 65536 ids: the one-read histogram with u16 LDS
    counters in segments of <= 65535 entries gives the checker's degrees — with a hub repeated
    more than 65535 times in one bucket, so counts cross the u16 range across segments."""
    import torch
    from sheep_amd import capi, device

    options(degree=2)
    rng = np.random.default_rng(7)
    n_ids = (1 << 26) - 5  # above 2^26 the bucketed path does not apply (global atomics)
    m = 1 << 21
    uv = rng.integers(0, n_ids, size=(m, 2)).astype(np.uint32)
    # 40 % of the records inside bucket 3: ~1.8 M endpoints counted in many 65535-entry folds
    dense = rng.random(m) < 0.4
    uv[dense] = (3 << 16) + rng.integers(0, 4000, size=(int(dense.sum()), 2)).astype(np.uint32)
    hub = rng.random(m) < 0.12  # ~250K occurrences of one id of bucket 3
    uv[hub, 0] = (3 << 16) + 17
    loops = rng.random(m) < 0.03
    uv[loops, 1] = uv[loops, 0]
    uv_d = torch.from_numpy(uv.view(np.int32)).cuda().view(torch.uint32)
    for mode in (capi.DEGREE_LLAMA, capi.DEGREE_FILE):
        got = device.degree(uv_d, n_ids, mode).cpu().numpy().view(np.uint32)
        want = oracle.degree(uv, mode, n_ids)
        assert np.array_equal(got, want)
        assert got[(3 << 16) + 17] > 65535


def test_graph2tree_all_self_loops_many_ids(oracle, gpu):
    """2^20 self-loop records over 200 000 ids (the hi-bin path with no estimated records):
    every vertex is an isolated root with pst 0; the bin cut must stay within its 512 slots."""
    import torch
    from sheep_amd import device

    m, n_ids = 1 << 20, 200000
    ids = np.random.default_rng(5).integers(0, n_ids, m).astype(np.uint32)
    uv = np.stack([ids, ids], axis=1)
    s_d, p_d, w_d, n = device.graph2tree(torch.from_numpy(uv.view(np.int32)).cuda().view(torch.uint32),
                                         n_ids)
    torch.cuda.synchronize()
    seq = oracle.degree_sequence(uv)
    p, w = oracle.build_tree(uv, seq)
    assert n == seq.size
    assert np.array_equal(s_d[:n].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(p_d[:n].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(w_d[:n].cpu().numpy().view(np.uint32), w)
    assert (p == 0xFFFFFFFF).all() and (w == 0).all()


@pytest.mark.parametrize("scale,k", [(0, 4), (14, 16), (16, 300)])
def test_partition_edges_writer_order(oracle, api, hep_edges, scale, k):
    """sheep_partition_edges (graph2tree -p K -o OUT on the GPU) against the reference's
    node-by-node writer restated in numpy: per part, the pairs (X < Y) in X order, then record
    order; self-loops skipped; the lower-sequence endpoint's part (partition.cpp:588-630)."""
    uv = hep_edges if scale == 0 else oracle.rmat(scale, 16, scale)
    seq = oracle.degree_sequence(uv)
    p, w = oracle.build_tree(uv, seq)
    parts = oracle.PartTree(p, w).partition(seq, k)
    got = api.partition_edges(uv, parts, seq)
    pos = np.full(parts.size, -1, np.int64)
    pos[seq] = np.arange(seq.size)
    x = uv.min(axis=1).astype(np.int64)
    y = uv.max(axis=1).astype(np.int64)
    keep = x != y
    idx = np.nonzero(keep)[0]
    owner = np.where(pos[x[idx]] < pos[y[idx]], parts[x[idx]], parts[y[idx]])
    order = np.lexsort((idx, x[idx], owner))  # by part, then X, then record
    assert len(got) == int(parts.max()) + 1
    at = 0
    for q, g in enumerate(got):
        sel = order[at:at + g.shape[0]]
        assert (owner[sel] == q).all()
        assert np.array_equal(g[:, 0], x[idx][sel]) and np.array_equal(g[:, 1], y[idx][sel])
        at += g.shape[0]
    assert at == idx.size


def test_dat_ingest_and_registered_records(oracle, api, tmp_path):
    """sheep_read_dat_dev / sheep_records_load_dat (pinned staging -> HBM, the f32 weight
    dropped) give the file's records for the whole file and every -l part, across the ingest's
    4M-record chunks; registered records give the same results as uploaded ones."""
    import ctypes

    import torch
    from sheep_amd import capi, device

    uv = oracle.rmat(18, 16, 5)  # 4.2 M records: two ingest chunks
    path = str(tmp_path / "r18.dat")
    api.write_dat(path, uv)
    got, mx = device.read_dat(path)
    assert np.array_equal(got.cpu().numpy().view(np.uint32), uv) and mx == int(uv.max()) + 1
    m = uv.shape[0]
    for part in (1, 2, 3):
        lo, hi = m * (part - 1) // 3, m * part // 3
        g, _ = device.read_dat(path, part, 3)
        assert np.array_equal(g.cpu().numpy().view(np.uint32), uv[lo:hi])
    host = np.zeros((m, 2), np.uint32)
    n = ctypes.c_uint64(0)
    capi.call("sheep_records_load_dat", path.encode(), 0, 0, ctypes.c_void_p(host.ctypes.data), m,
              ctypes.byref(n), None)
    try:
        assert np.array_equal(host, uv)
        seq = api.degree_sequence(host)  # through the registered device copy
        assert np.array_equal(seq, oracle.degree_sequence(uv))
        t = api.build_tree(host, seq)
        p, w = oracle.build_tree(uv, seq)
        assert np.array_equal(t.parent, p) and np.array_equal(t.pst, w)
    finally:
        capi.call("sheep_records_release", ctypes.c_void_p(host.ctypes.data))
    torch.cuda.synchronize()
