#!/usr/bin/env python3
"""Benchmark: edges/sec to build the elimination tree (BASELINE.json metric), MI355X.

One step = Sheep's timed window (graph2tree "Sorted" + "Mapped" [+ "Reduced"]) over one
synthetic R-MAT graph already resident in HBM as u32 (tail, head) pairs:
  degree histogram -> (degree, id) sort -> rank map -> edge pass -> tree build
  [N > 1: RCCL degree all-reduce, per-GPU partial trees, log2(N) merge to rank 0].
Workload: Graph500-style R-MAT scale 26, edgefactor 16 (1,073,741,824 records), seed 26 —
the metric's config (BASELINE.json configs[3]); it fits one GPU, so N=1 runs it whole and
N>1 shards the same records across ranks (strong scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S] [--no-cpu-baseline]
N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import platform
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md "HBM3E peak BW" (spec)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def pmc_traffic(kernel, key, field="hbm_bytes_per_launch_fetch_x2"):
    """HBM bytes per launch of `kernel` from the committed PMC summary (profiles/), if one was
    collected for this workload: FETCH_SIZE and WRITE_SIZE from separate rocprofv3 --pmc passes.
    The default field is the corrected one (MI355X_MICROARCH.md, HBM/rocprofv3: on gfx950
    FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so FETCH is doubled);
    "hbm_bytes_per_launch" is the raw FETCH + WRITE."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        tab = json.load(open(path))[key]
        base, _, targ = kernel.partition("<")  # "k_part<1>" matches "k_part<1, 512, 16>"
        byts = launches = 0
        for k, rec in tab.items():  # every template variant of the kernel (e.g. the map's hub one)
            kb, _, kt = k.replace("sheep::", "").partition("<")
            if kb == base and (not targ or kt.split(",")[0].rstrip(">").strip() == targ.rstrip(">")):
                n = rec.get("launches", 1)
                byts += rec[field] * n
                launches += n
        if launches:
            return byts / launches
    except (OSError, KeyError, ValueError):
        pass
    return None


def host_cpus():
    """The host's logical CPUs, those this process may run on, and its cgroup CPU quota."""
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(q) // int(per))
    except (OSError, ValueError):
        pass
    return {"logical": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "quota": quota,
            "model": cpu_model()}


def cpu_baseline(scale, edgefactor, seed):
    """Single-thread CPU restatement of graph2tree's Sorted+Mapped window (oracle, the
    reference's algorithm with FastUnionFind) on a bounded sample: R-MAT `scale`."""
    from oracle import oracle as O

    uv = O.rmat(scale, edgefactor, seed)
    sort_s, map_s, n_seq = O.time_graph2tree(uv, 1 << scale)
    m = uv.shape[0]
    return {"value": m / (sort_s + map_s), "unit": "edges/s", "cores": 1, "kind": "port",
            "sample": "R-MAT scale %d ef%d seed %d (%d records, %d non-isolated), sort %.3fs + "
                      "map %.3fs, CSR prebuilt (load excluded as in graph2tree), %s"
                      % (scale, edgefactor, seed, m, n_seq, sort_s, map_s, cpu_model())}


def cpu_baseline_ir(scale, edgefactor, seed, threads):
    """`mpirun -n T graph2tree -ir` analogue (the reference's multi-core CPU path): T record
    shards, mpiSequence, per-shard JTree, log2(T) merge reduce, on T host threads (oracle)."""
    from oracle import oracle as O

    uv = O.rmat(scale, edgefactor, seed)
    sort_s, map_s, red_s, n_seq, ok = O.time_graph2tree_ir(uv, 1 << scale, threads)
    m = uv.shape[0]
    return {"value": m / (sort_s + map_s + red_s), "unit": "edges/s", "cores": threads,
            "kind": "port", "exact": ok,
            "sample": "R-MAT scale %d ef%d seed %d (%d records), %d shards: sorted %.3fs + "
                      "mapped %.3fs + reduced %.3fs, %s" % (scale, edgefactor, seed, m, threads,
                                                           sort_s, map_s, red_s, cpu_model())}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="rmat", choices=["rmat", "lj", "twitter"],
                    help="rmat: Graph500 R-MAT (--scale); lj / twitter: the power-law configs "
                         "C3 / C5 of BASELINE.json")
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--seed", type=int, default=26)
    ap.add_argument("--cpu-scale", type=int, default=22)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify the tree against the CPU checker")
    # rehearsal of the N > 1 path on a one-GPU box (every rank on cuda:0, gloo carrying device
    # tensors: RCCL refuses two ranks on one device); timings are then meaningless
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--same-device", action="store_true")
    # N > 1: lockstep (the C++ driver sheep_graph2tree_multi_dev over its own RCCL communicator:
    # one kb loop walked by all ranks, kept pairs all-gathered per bucket), lockstep-py (the
    # same loop orchestrated from Python over torch.distributed; also the gloo / same-device
    # rehearsal) or merge (per-rank partial trees, gathered and merged on rank 0)
    ap.add_argument("--dist", default=os.environ.get("SHEEP_DIST", "lockstep"),
                    choices=["lockstep", "lockstep-py", "merge"])
    # N = 1 through the N > 1 code: the C++ multi-rank driver over a one-rank RCCL group, to
    # measure its host overhead and collective launches on one GPU (not the default N = 1 path)
    ap.add_argument("--lockstep-1", action="store_true")
    return ap.parse_args(argv)


# The rank setup below is shared by main() and tests/test_bench_ranks.py, which runs it over
# gloo process groups of 2 / 4 / 8 CPU ranks with the GPU calls stubbed (no 8-GPU node here).
def rank_env(gpus):
    """(world, rank, local) from the launcher's environment (torch.distributed.run)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (gpus, world))
    return world, rank, local


def load_shard(args, rank, world, dev):
    """This rank's contiguous record range [lo, hi) of the workload (graph2tree -l rank+1/world),
    generated in HBM by `dev` (sheep_amd.device): (uv, m, n_ids, lo, hi, workload, data)."""
    from sheep_amd.dist import shard_bounds

    scale, ef, seed = args.scale, args.edgefactor, args.seed
    if args.workload == "rmat":
        m = ef << scale
        n_ids = 1 << scale
        lo, hi = shard_bounds(m, rank, world)
        uv = dev.rmat(scale, ef, seed, lo, hi)  # this rank's records, resident in HBM
        wl = {"workload": "rmat%d_ef%d" % (scale, ef), "scale": scale, "edgefactor": ef,
              "seed": seed}
        data = "synthetic R-MAT (Graph500 A/B/C/D .57/.19/.19/.05), generated in HBM"
    else:
        n_ids, m, gamma, i0, seed = dev.POWERLAW[args.workload]
        lo, hi = shard_bounds(m, rank, world)
        uv = dev.powerlaw(n_ids, m, gamma, i0, seed, lo, hi)
        wl = {"workload": "%s_shape_powerlaw" % args.workload, "gamma": gamma, "i0": i0,
              "seed": seed}
        data = ("synthetic power-law (Chung-Lu, P(i) ~ (i+%g)^-1/(%g-1)), %s-shape n and m, "
                "generated in HBM" % (i0, gamma, args.workload))
    return uv, m, n_ids, lo, hi, wl, data


def native_driver(args, world):
    """Whether the step is the C++ multi-rank driver over its own RCCL communicator (the
    default for N > 1); the Python orchestration rehearses it where RCCL cannot run (gloo ranks
    sharing one device)."""
    return (world > 1 and args.dist == "lockstep" and args.backend == "nccl"
            and not args.same_device) or args.lockstep_1


def join_comm(rank, world, dev):
    """Rank 0 makes the RCCL id, the torch process group carries it to every rank, and each rank
    joins the library's communicator as (id, world, rank).  Returns the id."""
    uid = [dev.comm_unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(uid, src=0)
    dev.comm_init(uid[0], world, rank)
    return uid[0]


def main():
    args = parse_args()
    world, rank, local = rank_env(args.gpus)
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    if world > 1 or args.lockstep_1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    from sheep_amd import capi, device
    from sheep_amd.dist import DeviceOps, build_tree_lockstep, build_tree_sharded

    device.init(local)
    scale, ef, seed = args.scale, args.edgefactor, args.seed
    uv, m, n_ids, lo, hi, wl, data = load_shard(args, rank, world, device)
    torch.cuda.synchronize()
    ops = DeviceOps()
    native = native_driver(args, world)
    if world > 1 and args.dist == "lockstep" and not native:
        args.dist = "lockstep-py"
    if native:
        join_comm(rank, world, device)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def step():
        if native:
            return device.graph2tree_multi(uv, n_ids)
        if world == 1:
            return device.graph2tree(uv, n_ids)
        if args.dist == "lockstep-py":
            return build_tree_lockstep(uv, n_ids, ops)
        return build_tree_sharded(uv, n_ids, ops)

    for _ in range(args.warmup):
        out = step()
    barrier()
    phase = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
        # N > 1: the partial-tree build of this rank (the merge's own phases are "merge_*")
        tl = capi.last_timings()
        if world > 1 and args.dist == "merge" and not args.lockstep_1:
            tl = list(ops.build_timings) + [("merge_" + k, v) for k, v in tl]
        for name, ms in tl:
            phase.setdefault(name, []).append(ms)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    if rank == 0:
        ms_per_step = 1e3 * elapsed / args.steps
        n_seq = out[3] if world > 1 else out[3]
        value = m / (elapsed / args.steps)
        # Roofline of the dominant kernel: the one with the most time per step among the
        # kernels bracketed live by HIP events on the stream they run on.
        # "algo" is SURVEY §8(d)'s compulsory bytes attributed to the kernel: the degree pass's
        # one read of the records (k_front_fused / k_fh_count), the degree writes (the histogram), the rank/tree
        # pass's one read of the records plus the hi counts (k_kb_map); regrouping passes and
        # rank gathers count zero there.  "io" is the kernel's own streaming bytes (reads of its
        # input, writes of its output, 4 B per gathered rank), reported beside it.
        avg = {k: sum(v) / len(v) for k, v in phase.items()}
        recs = hi - lo if world > 1 else m
        key = "rmat%d" % scale if args.workload == "rmat" else args.workload
        # (kernel, phase, launches-phase or None, algo bytes per step, io bytes per step)
        table = [("k_kb_map", "kb_map", "kb_map#", 8 * recs + 4 * n_seq, 8 * recs + 4 * n_seq),
                 ("k_edge_bin", "edge_pass", None, 0, 20 * recs),
                 ("k_part<1>", "partition", None, 0, 20 * recs),
                 ("k_part<0>", "part_first", "part_first#", 0, 16 * recs),
                 ("k_front_fused", "front_fused", None, 8 * recs, 16 * recs),
                 ("k_fh_scatter", "degree_scatter", None, 0, 20 * recs),
                 ("k_fh_count", "degree_count", None, 8 * recs, 8 * recs),
                 ("k_degb_hist16", "degree_hist", None, 4 * n_ids, 4 * recs + 4 * n_ids)]
        cands = []
        for name, ph, nph, algo, io in table:
            if avg.get(ph):
                launches = avg[nph] if nph else 1
                if launches:
                    cands.append((name, avg[ph], launches, algo, io))
        roof = None
        if cands:
            name, ms, launches, algo, io = max(cands, key=lambda c: c[1])
            per_launch_ms = ms / launches
            ach = (algo / launches) / (per_launch_ms * 1e-3)
            roof = {"kernel": name, "bound": "hbm", "achieved": ach / 1e9,
                    "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": ach / HBM_PEAK,
                    "traffic": pmc_traffic(name, key), "algo_bytes": algo / launches,
                    "traffic_raw": pmc_traffic(name, key, "hbm_bytes_per_launch"),
                    "io_bytes": io / launches, "io_GB_s": io / (ms * 1e-3) / 1e9,
                    "avg_ms": per_launch_ms, "launches_per_step": launches,
                    "ms_per_step": ms,
                    "phases_ms": {k: round(v, 3) for k, v in avg.items() if not k.endswith("#")},
                    "others": {c[0]: {"ms_per_step": round(c[1], 3),
                                      "algo_GB_s": round(c[3] / (c[1] * 1e-3) / 1e9, 1),
                                      "io_GB_s": round(c[4] / (c[1] * 1e-3) / 1e9, 1),
                                      "traffic_per_launch": pmc_traffic(c[0], key)}
                               for c in cands if c[0] != name}}
        # SURVEY §8d B(m, n) = 16 m + 24 n with n = the id slots (its C4 row: 18.79 GB); the ids
        # of degree 0 are never touched by the sequence or the tree, so 24 n_seq is given beside
        path_bytes = 16 * m + 24 * n_ids
        label = "RMAT-%d" % scale if args.workload == "rmat" else wl["workload"]
        rec = {
            "metric": "edges/sec to build elimination tree (%s)" % label,
            "value": value, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u32",
            "data": data,
            "config": dict(wl, records=m, n_ids=n_ids, n_seq=n_seq,
                           parallelism=("edge-shard x%d (%s)" % (world, args.dist)
                                        if world > 1 else
                                        "lockstep driver, one-rank RCCL group" if args.lockstep_1
                                        else "single")),
            "path_roofline": {"bytes": path_bytes,
                              "frac": path_bytes / (elapsed / args.steps) / (world * HBM_PEAK),
                              "bytes_nseq": 16 * m + 24 * n_seq},
            "roofline": roof,
        }
        if args.check:
            rec["check"] = check_tree(out, uv if world == 1 else None, scale, ef, seed,
                                      args.workload)
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(args.cpu_scale, ef, args.cpu_scale)
            # `mpirun -n <cores>`: the cores this job may use — its cgroup CPU quota (the GPU
            # box: cpu.max 1600000/100000 = 16 of the host's 256 logical CPUs); more ranks than
            # that only time-slice inside the quota
            cpus = host_cpus()
            threads = cpus["quota"] or cpus["affinity"]
            rec["cpu_baseline_ir"] = cpu_baseline_ir(args.cpu_scale, ef, args.cpu_scale, threads)
            rec["cpu_baseline_ir"]["host_cpus"] = cpus
        print(json.dumps(rec), flush=True)
    if native:
        device.comm_free()
    if dist.is_initialized():
        dist.destroy_process_group()


def check_tree(out, uv_d, scale, ef, seed, workload):
    from oracle import oracle as O
    import numpy as np
    from sheep_amd import device

    seq_d, parent_d, pst_d, n = out[0], out[1], out[2], out[3]
    if workload == "rmat":
        uv = O.rmat(scale, ef, seed)
    else:
        uv = O.powerlaw(*device.POWERLAW[workload])
    seq = O.degree_sequence(uv)
    p, s = O.build_tree(uv, seq)
    ok = (n == len(seq)
          and np.array_equal(seq_d[:n].cpu().numpy().view(np.uint32), seq)
          and np.array_equal(parent_d[:n].cpu().numpy().view(np.uint32), p)
          and np.array_equal(pst_d[:n].cpu().numpy().view(np.uint32), s))
    return "bit-exact" if ok else "MISMATCH"


if __name__ == "__main__":
    main()
