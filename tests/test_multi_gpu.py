"""The multi-GPU driver (graph2tree -i -r, include/sheep_amd.h sheep_graph2tree_multi_*) against
the CPU checker, bit-exact.

RCCL refuses two ranks on one device, so the P-rank driver is run as P threads of one process
on cuda:0 (sheep_graph2tree_multi_local: the same C++ loop, its collectives as device copies),
and the RCCL communicator itself over a one-rank group (the code path of every rank of the
8-GPU run, collectives included)."""
import errno

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def shards_of(uv_d, P):
    from sheep_amd.dist import shard_bounds

    m = uv_d.shape[0]
    return [uv_d[shard_bounds(m, r, P)[0]:shard_bounds(m, r, P)[1]].contiguous() for r in range(P)]


def check(oracle, uv, mode, seq_d, parent_d, pst_d, n):
    seq = oracle.degree_sequence(uv, mode)
    p, w = oracle.build_tree(uv, seq)
    assert n == seq.size
    assert np.array_equal(seq_d[:n].cpu().numpy().view(np.uint32), seq)
    assert np.array_equal(parent_d[:n].cpu().numpy().view(np.uint32), p)
    assert np.array_equal(pst_d[:n].cpu().numpy().view(np.uint32), w)


@pytest.mark.parametrize("scale,seed,P,mode", [(12, 1, 1, 0), (16, 2, 2, 0), (16, 3, 3, 1),
                                               (18, 4, 4, 0), (18, 5, 8, 0), (19, 6, 8, 1)])
def test_multi_local_rmat(oracle, gpu, scale, seed, P, mode):
    import torch
    from sheep_amd import device

    uv_d = device.rmat(scale, 16, seed)
    torch.cuda.synchronize()
    out = device.graph2tree_multi_local(shards_of(uv_d, P), 1 << scale, mode)
    check(oracle, uv_d.cpu().numpy().view(np.uint32), mode, *out)


def test_multi_local_powerlaw_and_empty_shards(oracle, gpu):
    import torch
    from sheep_amd import device

    uv_d = device.powerlaw(300001, 2000000, 2.3, 100.0, 11)
    torch.cuda.synchronize()
    sh = shards_of(uv_d, 3)
    empty = uv_d[:0].contiguous()
    out = device.graph2tree_multi_local([sh[0], empty, sh[1], empty, sh[2]], 300001)
    check(oracle, uv_d.cpu().numpy().view(np.uint32), 0, *out)


def test_multi_local_hub_sequence_fallback(oracle, gpu):
    """The sharded sequence all-gathers P histograms over degree values: with a hub whose degree
    exceeds a rank's id slice it all-gathers the degree slices instead, same
    sequence.  4096 ids, P = 4 (slices of 1024 ids), hub degree ~3000."""
    import torch
    from sheep_amd import device

    rng = np.random.default_rng(7)
    hub = np.stack([np.zeros(3000, np.uint32), rng.integers(1, 4096, 3000).astype(np.uint32)], 1)
    rest = rng.integers(0, 4096, (20000, 2)).astype(np.uint32)
    uv = np.ascontiguousarray(rng.permutation(np.concatenate([hub, rest])))
    uv_d = torch.from_numpy(uv.view(np.int32)).cuda().view(torch.uint32)
    for P in (2, 4):
        out = device.graph2tree_multi_local(shards_of(uv_d, P), 4096)
        check(oracle, uv, 0, *out)


def test_multi_local_known_answer(oracle, gpu):
    import json
    import os

    import torch
    from conftest import GOLDEN
    from sheep_amd import device

    ka = np.array(json.load(open(os.path.join(GOLDEN, "known_answer.json")))["records"], np.uint32)
    uv_d = torch.from_numpy(ka.view(np.int32)).cuda().view(torch.uint32)
    out = device.graph2tree_multi_local([uv_d[i:i + 1].contiguous() for i in range(ka.shape[0])], 7)
    check(oracle, ka, 0, *out)


def test_rccl_one_rank_device_and_host(oracle, gpu, hep_edges):
    """The RCCL communicator path (unique id, init, the collectives) over a one-rank group:
    graph2tree_multi_dev, mpiSequence and the JTree + mpi_merge host entry."""
    import torch
    from sheep_amd import api, device

    uid = device.comm_unique_id()
    device.comm_init(uid, 1, 0)
    try:
        uv_d = device.rmat(18, 16, 9)
        out = device.graph2tree_multi(uv_d, 1 << 18)
        torch.cuda.synchronize()
        check(oracle, uv_d.cpu().numpy().view(np.uint32), 0, *out)
        seq = api.mpi_sequence(hep_edges, int(hep_edges.max()) + 1)
        assert np.array_equal(seq, oracle.degree_sequence(hep_edges))
        # a rank whose buffer is shorter than the global sequence (its share spans few ids):
        # -ERANGE with the global length, after the collectives; the retry then succeeds
        import ctypes
        from sheep_amd import capi
        small = np.zeros(4, np.uint32)
        n = ctypes.c_uint32(0)
        rc = capi.lib().sheep_mpi_sequence(api._ptr(hep_edges), hep_edges.shape[0], 0, 0,
                                           api._ptr(small), 4, ctypes.byref(n))
        assert rc == -errno.ERANGE and n.value == seq.size
        assert np.array_equal(api.mpi_sequence(hep_edges[:100]),
                              oracle.degree_sequence(hep_edges[:100]))
        t = api.build_tree_multi(hep_edges, seq)
        p, w = oracle.build_tree(hep_edges, seq)
        assert np.array_equal(t.parent, p) and np.array_equal(t.pst, w)
    finally:
        device.comm_free()


@pytest.mark.parametrize("env", [{"bin_slack": -900},               # every rank's bins overflow:
                                                                    # the scatter path per rank
                                 {"bin_direct": 0},                 # edge pass + bin scatter
                                 {"kb_gsum": 1},                    # the LDS giant summary
                                 {"part_overlap": 0},               # no first pass beside the degrees
                                 {"ls_split": 0},                   # every rank runs every zipper
                                 {"ls_seq": 0}])                    # every rank sorts all ids
def test_multi_local_front_half_options(oracle, gpu, options, env):
    """The multi-rank driver under the front-half / anchor options: the same tree (R-MAT 19,
    P = 2: 2^22 records per rank, so each rank runs the partitioned gathers)."""
    import torch
    from sheep_amd import device

    options(**env)
    uv_d = device.rmat(19, 16, 12)
    torch.cuda.synchronize()
    out = device.graph2tree_multi_local(shards_of(uv_d, 2), 1 << 19)
    check(oracle, uv_d.cpu().numpy().view(np.uint32), 0, *out)


def test_multi_local_one_rank_overflows(oracle, gpu):
    """Only one rank's direct bins overflow (its shard holds the records with the highest hi,
    far beyond its share of the global estimate): that rank groups its records through the
    scatter while the other stays direct; the tree is still the serial one."""
    import torch
    from sheep_amd import device

    uv_d = device.rmat(19, 16, 14)
    torch.cuda.synchronize()
    uv = uv_d.cpu().numpy().view(np.uint32)
    seq = oracle.degree_sequence(uv)
    rk = np.full(1 << 19, 0xFFFFFFFF, np.uint64)
    rk[seq] = np.arange(seq.size)
    hi = np.maximum(rk[uv[:, 0]], rk[uv[:, 1]])
    order = np.argsort(-hi.astype(np.int64), kind="stable")
    cut = uv.shape[0] // 10  # rank 0: the 10 % of records with the highest hi
    a = torch.from_numpy(np.ascontiguousarray(uv[order[:cut]]).view(np.int32)).cuda()
    b = torch.from_numpy(np.ascontiguousarray(uv[order[cut:]]).view(np.int32)).cuda()
    out = device.graph2tree_multi_local([a.view(torch.uint32), b.view(torch.uint32)], 1 << 19)
    check(oracle, uv, 0, *out)
