"""The multi-GPU driver (sheep_graph2tree_multi_dev, the code bench.py and `graph2tree -i -r`
run on every rank of an 8-GPU job) as P separate processes, the way torchrun / mpirun launch it.

RCCL refuses two ranks on one device, so on a one-GPU box the processes share cuda:0 and join
through the host shared-memory communicator (sheep_comm_init_host): the same C++ driver, each
process with its own HIP context and its own scratch, the collectives staged on the host.  It
covers what the P-thread rehearsal (test_multi_gpu.py) cannot: per-process state, the
all-gather and reduce-scatter layouts across processes, and every rank's copy of the result.
Bit-exact against the CPU checker."""
import uuid

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _u32(t, n):
    return t[:n].cpu().numpy().view(np.uint32).copy()


def _rank(r, world, name, scale, seed, opts, q, bad_rank=-1, digest_only=False):
    try:
        import torch

        from sheep_amd import capi, device
        from sheep_amd.dist import shard_bounds

        device.init(0)
        for k, v in opts.items():
            capi.set_option(k, v)
        m = 16 << scale
        lo, hi = shard_bounds(m, r, world)
        uv = device.rmat(scale, 16, seed, lo, hi)
        if r == bad_rank:  # one record of this shard names an id past the id space
            uv.view(torch.int32)[7, 1] = (1 << scale) + 5
        torch.cuda.synchronize()
        device.comm_init_host(name, world, r)
        try:
            try:
                seq, parent, pst, n = device.graph2tree_multi(uv, 1 << scale)
                torch.cuda.synchronize()
            except capi.SheepError as e:
                q.put((r, 0, None, None, None, ("code", e.code)))
                return
            phases = [k for k, _ in capi.last_timings()]
            if digest_only:
                q.put((r, n, _h16(seq, n), _h16(parent, n), _h16(pst, n), ("phases", phases)))
            else:
                q.put((r, n, _u32(seq, n), _u32(parent, n), _u32(pst, n), ("phases", phases)))
        finally:
            device.comm_free()
    except Exception as e:  # reported to the parent (a failing rank leaves the others waiting)
        q.put((r, 0, None, None, None, repr(e)))


def _h16(t, n):
    import hashlib

    return hashlib.sha256(_u32(t, n).view(np.uint8)).hexdigest()[:16]


def _run_ranks(world, scale, seed, opts, bad_rank=-1, digest_only=False, timeout=240):
    """Start `world` spawned ranks of _rank and collect their results; ranks left behind (a
    failed one leaves the others in a collective) are ended."""
    q = mp.get_context("spawn").Queue()
    name = "/sheep-test-%s" % uuid.uuid4().hex[:16]
    pc = mp.start_processes(_rank, args=(world, name, scale, seed, opts, q, bad_rank, digest_only),
                            nprocs=world, join=False, start_method="spawn")
    got = {}
    try:
        for _ in range(world):
            r, n, seq, parent, pst, info = q.get(timeout=timeout)
            got[r] = (n, seq, parent, pst, info)
        while not pc.join(timeout=60):
            pass
    finally:
        for proc in pc.processes:
            if proc.is_alive():
                proc.kill()
    return got


@pytest.mark.parametrize("world,scale,seed,opts", [
    (2, 16, 41, {}),
    (3, 17, 42, {}),                              # three ranks: uneven id slices
    (4, 16, 43, {"ls_split": 0, "ls_seq": 0}),    # replicated apply, all-reduced degrees
    (8, 16, 44, {}),                              # the headline's P: 8 processes, 8 id slices
])
def test_multi_process_host_comm(oracle, world, scale, seed, opts):
    got = _run_ranks(world, scale, seed, opts)
    for r in range(world):
        assert got[r][4][0] == "phases", "rank %d: %s" % (r, got[r][4])
    uv = oracle.rmat(scale, 16, seed)
    oseq = oracle.degree_sequence(uv)
    p, s = oracle.build_tree(uv, oseq)
    for r in range(world):  # every rank holds the whole tree
        n, seq, parent, pst, _ = got[r]
        assert n == oseq.size
        assert np.array_equal(seq, oseq)
        assert np.array_equal(parent, p)
        assert np.array_equal(pst, s)


@pytest.mark.parametrize("ls_seq", [1, 0])
def test_multi_process_range_error_on_every_rank(ls_seq):
    """One rank's shard holds an id >= n_ids (index.at(), jtree.cpp:75): EVERY rank returns
    -ERANGE after the same collectives, none hangs (the check after the sequence
    and after the edge pass was local, so the failing rank threw while its peers waited in the
    next all-reduce).  Both sequence paths: sharded (1) and all-reduced (0)."""
    import errno

    got = _run_ranks(2, 16, 45, {"ls_seq": ls_seq}, bad_rank=1, timeout=180)
    for r in range(2):
        assert got[r][4] == ("code", -errno.ERANGE), "rank %d: %s" % (r, got[r][4])


def test_multi_process_fused_front_half():
    """C2 (R-MAT 22, seed 22) as 2 processes of 2^25 records each: every rank's front half
    takes the fused one-read pass (launch_front_fused into sampled capacity regions, what
    graph2tree_dev runs at that size), and every rank's seq / parent / pst equal the checker's
    committed digests (tests/golden/digests.json)."""
    import json
    import os

    from conftest import GOLDEN

    d = json.load(open(os.path.join(GOLDEN, "digests.json")))["c2_rmat22"]
    assert (d["scale"], d["seed"]) == (22, 22)
    got = _run_ranks(2, 22, 22, {}, digest_only=True)
    for r in range(2):
        n, hs, hp, hw, info = got[r]
        assert info[0] == "phases", "rank %d: %s" % (r, info)
        assert "front_fused" in info[1] and "degree_exact" not in info[1], info[1]
        assert n == d["n_seq"]
        assert (hs, hp, hw) == (d["seq"], d["parent"], d["pst"])


def _seq_rank(r, world, name, shards, q):
    try:
        from sheep_amd import api, device

        device.init(0)
        device.comm_init_host(name, world, r)
        try:
            q.put((r, api.mpi_sequence(shards[r]), None))
        finally:
            device.comm_free()
    except Exception as e:
        q.put((r, None, repr(e)))


def test_mpi_sequence_retry_on_every_rank(oracle):
    """mpiSequence (sequence.h:65-93) where rank 0's records span only ids 0..15: its buffer
    (max id + 1) is shorter than the global sequence, so EVERY rank gets -ERANGE with the global
    length and every rank must retry, including rank 1, whose buffer was large enough (ADVICE
    r03: it used to raise while rank 0 retried alone and waited forever)."""
    rng = np.random.default_rng(5)
    small = rng.integers(0, 16, (200, 2)).astype(np.uint32)
    large = rng.integers(0, 5000, (20000, 2)).astype(np.uint32)
    q = mp.get_context("spawn").Queue()
    name = "/sheep-test-%s" % uuid.uuid4().hex[:16]
    pc = mp.start_processes(_seq_rank, args=(2, name, [small, large], q), nprocs=2, join=False,
                            start_method="spawn")
    got = {}
    try:
        for _ in range(2):
            r, seq, err = q.get(timeout=180)
            assert err is None, "rank %d: %s" % (r, err)
            got[r] = seq
        while not pc.join(timeout=60):
            pass
    finally:
        for proc in pc.processes:
            if proc.is_alive():
                proc.kill()
    want = oracle.degree_sequence(np.concatenate([small, large]))
    assert want.size > 16
    for r in range(2):
        assert np.array_equal(got[r], want)
