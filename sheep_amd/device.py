"""Device-resident hot path: torch owns HBM buffers and streams, libsheep_amd.so does the work.

Every function takes torch tensors on a ``cuda`` (HIP) device and enqueues on torch's current
stream, so it composes with torch.distributed (RCCL) collectives on the same stream.
"""
import ctypes

import torch

from . import capi


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def init(device_index):
    capi.call("sheep_gpu_init", int(device_index))


def rmat(scale, edgefactor, seed, e_begin=0, e_end=None, device="cuda"):
    """R-MAT records [e_begin, e_end) of the (scale, seed) stream as an (n, 2) uint32 tensor."""
    m = edgefactor << scale
    if e_end is None:
        e_end = m
    uv = torch.empty((e_end - e_begin, 2), dtype=torch.uint32, device=device)
    capi.call("sheep_rmat_dev", _p(uv), scale, seed, e_begin, e_end, _stream())
    return uv


# Power-law workloads (BASELINE.json configs C3, C5): (n ids, m records, gamma, i0, seed)
POWERLAW = {
    "lj": (4847571, 68993773, 2.3, 100.0, 3),
    "twitter": (41652230, 1468365182, 2.1, 50.0, 5),
}


def powerlaw(n, m, gamma, i0, seed, e_begin=0, e_end=None, device="cuda"):
    """Power-law records [e_begin, e_end) of the (n, gamma, i0, seed) stream, (k, 2) uint32."""
    if e_end is None:
        e_end = m
    uv = torch.empty((e_end - e_begin, 2), dtype=torch.uint32, device=device)
    capi.call("sheep_powerlaw_dev", _p(uv), n, float(gamma), float(i0), seed, e_begin, e_end,
              _stream())
    return uv


def degree(uv, n_ids, mode=capi.DEGREE_LLAMA, out=None):
    deg = out if out is not None else torch.empty(n_ids, dtype=torch.uint32, device=uv.device)
    capi.call("sheep_degree_dev", _p(uv), uv.shape[0], n_ids, mode, _p(deg), _stream())
    return deg


def degree_ex(uv, n_ids, mode=capi.DEGREE_LLAMA):
    """(deg, selfc): degrees and self-loop record counts of these records."""
    deg = torch.empty(max(n_ids, 1), dtype=torch.uint32, device=uv.device)
    selfc = torch.empty(max(n_ids, 1), dtype=torch.uint32, device=uv.device)
    capi.call("sheep_degree_ex_dev", _p(uv), uv.shape[0], n_ids, mode, _p(deg), _p(selfc),
              _stream())
    return deg[:n_ids], selfc[:n_ids]


def build_tree_deg(uv, rank, seq, n_seq, deg, selfc, mode=capi.DEGREE_LLAMA):
    """build_tree with pst derived from these records' own degrees (no per-edge atomics)."""
    parent = torch.empty(max(n_seq, 1), dtype=torch.uint32, device=uv.device)
    pst = torch.empty(max(n_seq, 1), dtype=torch.uint32, device=uv.device)
    capi.call("sheep_build_tree_deg_dev", _p(uv), uv.shape[0], _p(rank), rank.numel(), _p(seq),
              n_seq, _p(deg), _p(selfc), mode, _p(parent), _p(pst), _stream())
    return parent, pst


def sequence(deg, seq=None, rank=None):
    n_ids = deg.numel()
    seq = seq if seq is not None else torch.empty(max(n_ids, 1), dtype=torch.uint32, device=deg.device)
    rank = rank if rank is not None else torch.empty(max(n_ids, 1), dtype=torch.uint32,
                                                     device=deg.device)
    n_seq = ctypes.c_uint32(0)
    capi.call("sheep_sequence_dev", _p(deg), n_ids, _p(seq), _p(rank), ctypes.byref(n_seq),
              _stream())
    return seq, rank, n_seq.value


def build_tree(uv, rank, n_seq, parent=None, pst=None):
    parent = parent if parent is not None else torch.empty(max(n_seq, 1), dtype=torch.uint32,
                                                           device=uv.device)
    pst = pst if pst is not None else torch.empty(max(n_seq, 1), dtype=torch.uint32, device=uv.device)
    capi.call("sheep_build_tree_dev", _p(uv), uv.shape[0], _p(rank), rank.numel(), n_seq,
              _p(parent), _p(pst), _stream())
    return parent, pst


def merge_into(parent_a, pst_a, parent_b, pst_b, n):
    """(parent_a, pst_a) <- etree(A ∪ B), in place."""
    capi.call("sheep_merge_trees_dev", _p(parent_a), _p(pst_a), _p(parent_b), _p(pst_b), n,
              _stream())


def merge_forests(parents, n, out=None):
    """etree of the union of the forests in ``parents`` ((T, >= n) uint32, INVALID = root)."""
    T = parents.shape[0]
    parents = parents[:, :n].contiguous()
    out = out if out is not None else torch.empty(max(n, 1), dtype=torch.uint32,
                                                  device=parents.device)
    capi.call("sheep_merge_forests_dev", _p(parents), T, n, _p(out), _stream())
    return out


class Lockstep:
    """One rank's side of the lockstep multi-GPU tree build (sheep_ls_*, include/sheep_amd.h).
    The collectives are the caller's (sheep_amd.dist.build_tree_lockstep)."""

    def __init__(self, uv, rank, seq, n_seq, deg):
        import numpy as np

        self.m = uv.shape[0]
        self.n_seq = n_seq
        counts = np.zeros(513, np.uint64)
        nb = ctypes.c_uint32(0)
        h = ctypes.c_void_p()
        capi.call("sheep_ls_begin", _p(uv), self.m, _p(rank), rank.numel(), _p(seq), n_seq,
                  _p(deg), ctypes.c_void_p(counts.ctypes.data), ctypes.byref(nb),
                  ctypes.byref(h), _stream())
        self.h = h
        self.bin_counts = counts[:nb.value].astype(np.int64)

    def plan(self, global_counts):
        """global_counts: this shard's bin_counts summed over ranks -> (buckets, mark slots)."""
        import numpy as np

        g = np.ascontiguousarray(np.asarray(global_counts, dtype=np.uint64))
        nbk, ms = ctypes.c_uint32(0), ctypes.c_uint32(0)
        capi.call("sheep_ls_plan", self.h, ctypes.c_void_p(g.ctypes.data), ctypes.byref(nbk),
                  ctypes.byref(ms))
        self.slots = ms.value
        return nbk.value, ms.value

    def split(self, rank, n_ranks):
        """Split apply (n_ranks >= 2): this rank runs the zipper of buckets k = rank mod P only;
        finish() then returns its buckets' forest edges (the ranks' forests are disjoint)."""
        capi.call("sheep_ls_split", self.h, rank, n_ranks)

    def map(self, k, send, count=None):
        """Map bucket k into send; with ``count`` (cuda int64 tensor) the kept-pair count is
        written there (no synchronisation) and None returned, else it is returned."""
        if count is not None:
            capi.call("sheep_ls_map", self.h, k, _p(send), _p(count), None, _stream())
            return None
        n = ctypes.c_uint32(0)
        capi.call("sheep_ls_map", self.h, k, _p(send), None, ctypes.byref(n), _stream())
        return n.value

    def pack(self, k, send, cap):
        capi.call("sheep_ls_pack", self.h, k, _p(send), cap, _stream())

    def apply(self, k, recv, n_ranks, cap):
        capi.call("sheep_ls_apply", self.h, k, _p(recv), n_ranks, cap, _stream())

    def finish(self, seq, deg_local, selfc, mode=capi.DEGREE_LLAMA):
        dev = seq.device
        parent = torch.empty(max(self.n_seq, 1), dtype=torch.uint32, device=dev)
        pst = torch.empty(max(self.n_seq, 1), dtype=torch.uint32, device=dev)
        capi.call("sheep_ls_finish", self.h, _p(seq), _p(deg_local), _p(selfc), mode, _p(parent),
                  _p(pst), _stream())
        return parent, pst

    def free(self):
        if self.h:
            capi.call("sheep_ls_free", self.h)
            self.h = None


EVAL_KEYS = ("edges_cut", "vcom_vol", "vertex_bal", "ecv_hash", "hash_bal", "ecv_down",
             "down_bal", "ecv_up", "up_bal", "edges", "nodes")


def evaluate(uv, parts, rank, n_parts=None):
    """Partition::evaluate(graph, seq) on the GPU: ``parts`` int16 per vertex id (cuda),
    ``rank`` the positions in seq (sheep_sequence_dev).  Returns a dict (EVAL_KEYS)."""
    import numpy as np

    if n_parts is None:
        n_parts = int(parts.max().item()) + 1
    out = np.zeros(11, np.uint64)
    capi.call("sheep_evaluate_dev", _p(uv), uv.shape[0], _p(parts), _p(rank), parts.numel(),
              n_parts, ctypes.c_void_p(out.ctypes.data), _stream())
    return dict(zip(EVAL_KEYS, (int(x) for x in out)))


def graph2tree(uv, n_ids, mode=capi.DEGREE_LLAMA, seq=None, parent=None, pst=None):
    dev = uv.device
    seq = seq if seq is not None else torch.empty(max(n_ids, 1), dtype=torch.uint32, device=dev)
    parent = parent if parent is not None else torch.empty(max(n_ids, 1), dtype=torch.uint32, device=dev)
    pst = pst if pst is not None else torch.empty(max(n_ids, 1), dtype=torch.uint32, device=dev)
    n_seq = ctypes.c_uint32(0)
    capi.call("sheep_graph2tree_dev", _p(uv), uv.shape[0], n_ids, mode, _p(seq), _p(parent),
              _p(pst), ctypes.byref(n_seq), _stream())
    return seq, parent, pst, n_seq.value


# ---- multi-GPU (graph2tree -i -r over RCCL; include/sheep_amd.h) -------------------------------

def comm_unique_id():
    """128-byte RCCL id (rank 0 makes it; every rank passes it to comm_init)."""
    buf = ctypes.create_string_buffer(128)
    capi.call("sheep_comm_unique_id", ctypes.cast(buf, ctypes.c_void_p))
    return buf.raw


def comm_init(uid, n_ranks, rank):
    buf = ctypes.create_string_buffer(bytes(uid), 128)
    capi.call("sheep_comm_init", ctypes.cast(buf, ctypes.c_void_p), int(n_ranks), int(rank))


def comm_init_host(name, n_ranks, rank):
    """The group through host shared memory (sheep_comm_init_host): P processes on one GPU."""
    capi.call("sheep_comm_init_host", name.encode(), int(n_ranks), int(rank))


def comm_free():
    capi.call("sheep_comm_free")


def graph2tree_multi(uv, n_ids, mode=capi.DEGREE_LLAMA):
    """This rank's shard -> (seq, parent, pst, n_seq) of the whole graph, on every rank."""
    dev = uv.device
    out = [torch.empty(max(n_ids, 1), dtype=torch.uint32, device=dev) for _ in range(3)]
    n_seq = ctypes.c_uint32(0)
    capi.call("sheep_graph2tree_multi_dev", _p(uv), uv.shape[0], n_ids, mode, _p(out[0]),
              _p(out[1]), _p(out[2]), ctypes.byref(n_seq), _stream())
    return out[0], out[1], out[2], n_seq.value


def graph2tree_multi_local(shards, n_ids, mode=capi.DEGREE_LLAMA):
    """The P-rank driver with P shards on this device (one thread per rank): rank 0's result."""
    P = len(shards)
    dev = shards[0].device
    ptrs = (ctypes.c_void_p * P)(*[s.data_ptr() for s in shards])
    ms = (ctypes.c_uint64 * P)(*[s.shape[0] for s in shards])
    out = [torch.empty(max(n_ids, 1), dtype=torch.uint32, device=dev) for _ in range(3)]
    n_seq = ctypes.c_uint32(0)
    torch.cuda.synchronize()
    capi.call("sheep_graph2tree_multi_local", ctypes.cast(ptrs, ctypes.c_void_p),
              ctypes.cast(ms, ctypes.c_void_p), P, n_ids, mode, _p(out[0]), _p(out[1]), _p(out[2]),
              ctypes.byref(n_seq))
    return out[0], out[1], out[2], n_seq.value


def read_dat(path, part=0, num_parts=0, device="cuda"):
    """XS1 records of a .dat file (or the part/num_parts range, 1-based as graph2tree -l)
    straight into HBM through pinned staging: (uv (m, 2) uint32 tensor, max id + 1)."""
    m = ctypes.c_uint64(0)
    capi.call("sheep_read_dat_dev", str(path).encode(), part, num_parts, None, 0, ctypes.byref(m),
              None, _stream())
    uv = torch.empty((max(m.value, 1), 2), dtype=torch.uint32, device=device)
    mx = ctypes.c_uint32(0)
    capi.call("sheep_read_dat_dev", str(path).encode(), part, num_parts, _p(uv), m.value,
              ctypes.byref(m), ctypes.byref(mx), _stream())
    return uv[:m.value], mx.value
