"""bench.py's N > 1 rank setup on CPU, without GPUs.

The driver launches `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`
on an 8-GPU node, which this pool never gives us.  These tests run bench.py's own rank setup —
rank_env (WORLD_SIZE / RANK / LOCAL_RANK), load_shard (each rank's contiguous record range,
graph2tree -l r+1/N), native_driver (the C++ multi-rank driver over RCCL is the default) and
join_comm (rank 0's RCCL id broadcast over the torch process group, then comm_init(id, N, r)) —
in N CPU processes over a gloo group, for N = 2, 4, 8, with the GPU calls replaced by a
recording stand-in at the Python level.  What it pins: every rank reaches
sheep_graph2tree_multi_dev's communicator with the same id and its own (N, rank), on the
device LOCAL_RANK, and the shards tile the headline workload exactly.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import json, os, sys
sys.path.insert(0, sys.argv[1])
import torch.distributed as dist
import bench

from sheep_amd.device import POWERLAW  # (the workload table; no GPU call)

class FakeDevice:
    POWERLAW = POWERLAW
    def __init__(self):
        self.calls = []
    def rmat(self, scale, ef, seed, lo, hi):
        self.calls.append(["rmat", scale, ef, seed, lo, hi])
        return ("records", lo, hi)
    def powerlaw(self, n, m, gamma, i0, seed, lo, hi):
        self.calls.append(["powerlaw", n, m, lo, hi])
        return ("records", lo, hi)
    def comm_unique_id(self):
        self.calls.append(["comm_unique_id"])
        return os.urandom(128)
    def comm_init(self, uid, n, r):
        self.calls.append(["comm_init", bytes(uid).hex(), n, r])

argv = sys.argv[3:]
args = bench.parse_args(argv)
world, rank, local = bench.rank_env(args.gpus)
dist.init_process_group("gloo")  # (the product path uses "nccl" with device_id=cuda:local)
dev = FakeDevice()
uv, m, n_ids, lo, hi, wl, data = bench.load_shard(args, rank, world, dev)
native = bench.native_driver(args, world)
uid = bench.join_comm(rank, world, dev).hex() if native else None
rec = {"rank": rank, "world": world, "local": local, "m": m, "n_ids": n_ids, "lo": lo, "hi": hi,
       "native": native, "uid": uid, "calls": dev.calls, "workload": wl["workload"]}
out = [None] * world
dist.all_gather_object(out, rec)
if rank == 0:
    with open(sys.argv[2], "w") as f:
        json.dump(out, f)
dist.destroy_process_group()
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, tmp_path, extra=()):
    port = _free_port()
    out = tmp_path / ("ranks%d.json" % world)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER, ROOT, str(out),
                                       "--gpus", str(world)] + list(extra), env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace"))
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)[-3000:]
    return json.load(open(out))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_rank_setup_rmat26(world, tmp_path):
    recs = _run(world, tmp_path)
    assert [r["rank"] for r in recs] == list(range(world))
    m = 16 << 26
    # the shards tile RMAT-26's records contiguously, within one record of m / N each
    assert recs[0]["lo"] == 0 and recs[-1]["hi"] == m
    for a, b in zip(recs, recs[1:]):
        assert a["hi"] == b["lo"]
    assert max(r["hi"] - r["lo"] for r in recs) - min(r["hi"] - r["lo"] for r in recs) <= 1
    for r in recs:
        assert r["m"] == m and r["n_ids"] == 1 << 26 and r["world"] == world
        assert r["local"] == r["rank"]  # torch.cuda.set_device(LOCAL_RANK)
        assert r["native"]  # the C++ driver over RCCL is the default N > 1 step
        assert r["calls"][0] == ["rmat", 26, 16, 26, r["lo"], r["hi"]]
    # one id, made on rank 0 only, joined by every rank as (id, N, rank)
    uid = recs[0]["uid"]
    assert len(uid) == 256 and all(r["uid"] == uid for r in recs)
    assert ["comm_unique_id"] in recs[0]["calls"]
    for r in recs:
        assert (["comm_unique_id"] in r["calls"]) == (r["rank"] == 0)
        assert r["calls"][-1] == ["comm_init", uid, world, r["rank"]]


def test_bench_rank_setup_twitter_and_rehearsal(tmp_path):
    """The power-law config shards the same way; the gloo rehearsal (--backend gloo) takes the
    Python orchestration instead of the native driver, so nothing joins RCCL."""
    recs = _run(4, tmp_path, ["--workload", "twitter", "--backend", "gloo"])
    m = 1468365182
    assert recs[0]["lo"] == 0 and recs[-1]["hi"] == m
    for a, b in zip(recs, recs[1:]):
        assert a["hi"] == b["lo"]
    for r in recs:
        assert not r["native"] and r["uid"] is None
        assert r["calls"] == [["powerlaw", 41652230, m, r["lo"], r["hi"]]]


def test_rank_env_refuses_mismatch(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench

    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert bench.rank_env(8) == (8, 3, 3)
    with pytest.raises(SystemExit):
        bench.rank_env(4)
