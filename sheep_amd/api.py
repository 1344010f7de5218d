"""The reference's lib/ interface over the MI355X C-ABI.

Names and argument meaning follow arpang/sheep lib/:
  degree_sequence(edges)        lib/sequence.h:52-63   (LLAMA degrees, graph2tree's default)
  file_sequence(path)           lib/sequence.h:95-128  (degree_sequence binary: FILE degrees
                                                         over the XS1Reader / SNAPReader stream)
  build_tree(edges, seq)        lib/jtree.h:111-136    (JTree(graph, seq) -> jnodes)
  merge_trees(a, b)             lib/jnode.cpp:174-201  (JNodeTable::merge)
  read_dat / read_net           lib/readerwriter.h:42-90 and LLAMA's .dat loader
  write_sequence/read_sequence  lib/sequence.h:153-184 (text, one id per line)
  JNodeTable.save / load        lib/jnode.cpp:52-102,164-168 (.tre: u32 end_id + n x {parent,pst})
Errors raise SheepError (the reference throws / asserts: see include/sheep_amd.h).
"""
import ctypes
import errno

import numpy as np

from . import capi
from .capi import DEGREE_FILE, DEGREE_LLAMA, INVALID, SheepError  # noqa: F401

_XS1 = np.dtype([("tail", "<u4"), ("head", "<u4"), ("weight", "<f4")])


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None and a.size else None


# ---- edge files ------------------------------------------------------------------------------

def read_dat(path):
    """All complete 12-byte XS1 records as an (m, 2) uint32 array (LLAMA's .dat load)."""
    raw = np.fromfile(path, dtype=np.uint8)
    m = raw.size // 12
    return np.ascontiguousarray(raw[: m * 12].view(_XS1)[["tail", "head"]]
                                .view(np.uint32).reshape(m, 3)[:, :2])


def read_dat_stream(path):
    """The XS1Reader record stream (readerwriter.h:50-58): eof() is tested before read(), so
    the final failed read returns the previous record again -> the last record appears twice."""
    uv = read_dat(path)
    if uv.shape[0]:
        uv = np.concatenate([uv, uv[-1:]])
    return uv


def read_net(path):
    """SNAPReader (readerwriter.h:84-89): whitespace-separated unsigned pairs, stopping at the
    first token that is not an unsigned integer (e.g. a '#' comment)."""
    vals = []
    with open(path) as f:
        for tok in f.read().split():
            if not tok.isdigit() or int(tok) > 0xFFFFFFFF:
                break
            vals.append(int(tok))
    vals = vals[: len(vals) // 2 * 2]
    return np.array(vals, dtype=np.uint32).reshape(-1, 2)


def write_dat(path, uv):
    """XS1Writer (readerwriter.h:61-76): weight 1.0 on every record."""
    rec = np.zeros(uv.shape[0], _XS1)
    rec["tail"], rec["head"], rec["weight"] = uv[:, 0], uv[:, 1], 1.0
    rec.tofile(path)


def read_edges(path):
    """graph2tree's load of a graph file (LLAMA: .dat binary, else SNAP text)."""
    return read_dat(path) if path.endswith(".dat") else read_net(path)


# ---- sequences -------------------------------------------------------------------------------

def _as_edges(uv):
    uv = np.ascontiguousarray(uv, dtype=np.uint32)
    if uv.ndim != 2 or uv.shape[1] != 2:
        uv = uv.reshape(-1, 2)
    return uv


def degree_sequence(uv, mode=DEGREE_LLAMA, n_ids=0, return_rank=False):
    uv = _as_edges(uv)
    m = uv.shape[0]
    if n_ids == 0 and m:
        n_ids = int(uv.max()) + 1
    seq = np.zeros(max(n_ids, 1), np.uint32)
    rank = np.zeros(max(n_ids, 1), np.uint32) if return_rank else None
    n_seq = ctypes.c_uint32(0)
    if m:
        capi.call("sheep_degree_seq", _ptr(uv), m, n_ids, mode, _ptr(seq),
                  ctypes.byref(n_seq), _ptr(rank))
    seq = seq[: n_seq.value].copy()
    return (seq, rank[:n_ids]) if return_rank else seq


def file_sequence(path):
    """fileSequence (sequence.h:124-128): FILE-mode degrees over the reader stream."""
    uv = read_dat_stream(path) if path.endswith(".dat") else read_net(path)
    return degree_sequence(uv, DEGREE_FILE)


def write_sequence(seq, path):
    with open(path, "w") as f:
        f.write("".join("%d\n" % x for x in seq))


def read_sequence(path):
    with open(path) as f:
        vals = []
        for tok in f.read().split():
            if not tok.isdigit():
                break
            vals.append(int(tok))
    return np.array(vals, dtype=np.uint32)


# ---- trees -----------------------------------------------------------------------------------

class JNodeTable:
    """parent / pst_weight per jnid (jnode.h:56-69), INVALID parent = root."""

    def __init__(self, parent, pst):
        self.parent = np.ascontiguousarray(parent, np.uint32)
        self.pst = np.ascontiguousarray(pst, np.uint32)

    def size(self):
        return int(self.parent.size)

    def save(self, path):
        """.tre: u32 end_id, then max_id x {u32 parent, u32 pst_weight} (jnode.cpp:164-168)."""
        body = np.empty((self.size(), 2), np.uint32)
        body[:, 0], body[:, 1] = self.parent, self.pst
        with open(path, "wb") as f:
            f.write(np.uint32(self.size()).tobytes())
            f.write(body.tobytes())

    @classmethod
    def load(cls, path):
        """Open constructor (jnode.cpp:76-102): max_id from the file size, end_id from header."""
        raw = np.fromfile(path, dtype=np.uint32)
        end_id = int(raw[0])
        body = raw[1:].reshape(-1, 2)[:end_id]
        return cls(body[:, 0].copy(), body[:, 1].copy())

    def merge(self, other):
        return merge_trees(self, other)

    def __eq__(self, o):
        return np.array_equal(self.parent, o.parent) and np.array_equal(self.pst, o.pst)


def build_tree(uv, seq):
    """JTree(graph, seq).jnodes on the GPU."""
    uv = _as_edges(uv)
    seq = np.ascontiguousarray(seq, np.uint32)
    n = seq.size
    parent = np.zeros(max(n, 1), np.uint32)
    pst = np.zeros(max(n, 1), np.uint32)
    if n:
        capi.call("sheep_build_tree", _ptr(uv), uv.shape[0], _ptr(seq), n, _ptr(parent), _ptr(pst))
    return JNodeTable(parent[:n], pst[:n])


def merge_trees(a, b):
    if a.size() != b.size():
        raise SheepError(-22, "merge: trees of different sizes (jnode.cpp:176)")
    n = a.size()
    parent = np.zeros(max(n, 1), np.uint32)
    pst = np.zeros(max(n, 1), np.uint32)
    if n:
        capi.call("sheep_merge_trees", _ptr(a.parent), _ptr(a.pst), _ptr(b.parent), _ptr(b.pst), n,
                  _ptr(parent), _ptr(pst))
    return JNodeTable(parent[:n], pst[:n])


def graph2tree(uv, mode=DEGREE_LLAMA):
    """graph2tree's serial path (graph2tree.cpp:162-193): degreeSequence + JTree."""
    seq = degree_sequence(uv, mode)
    return seq, build_tree(uv, seq)


# ---- partition (host, as in the reference) ---------------------------------------------------

def partition(tree, seq, ks, balance=1.03):
    """Partition(seq, jnodes, k, balance) (partition.cpp:50-67 -> forwardPartition :86-157) for
    each k of ``ks`` in turn on ONE table, as partition_tree runs its k list.  Returns a list of
    vid-indexed int16 part arrays (-1 for ids not in seq) and the created part counts."""
    seq = np.ascontiguousarray(seq, np.uint32)
    ks = np.ascontiguousarray(np.atleast_1d(ks), np.int32)
    n_vid = int(seq.max()) + 1 if seq.size else 0
    parts = np.empty((ks.size, max(n_vid, 1)), np.int16)
    created = np.zeros(ks.size, np.uint32)
    capi.call("sheep_partition", _ptr(tree.parent), _ptr(tree.pst), tree.size(), _ptr(seq),
              _ptr(ks), ks.size, float(balance), _ptr(parts), n_vid, _ptr(created))
    return [parts[i, :n_vid] for i in range(ks.size)], [int(c) for c in created]


# ---- multi-rank (graph2tree -i -r; a communicator from sheep_comm_init on every rank) ---------

def mpi_sequence(uv, n_ids=0, mode=DEGREE_LLAMA):
    """mpiSequence (sequence.h:65-93): this rank's records; the same sequence on every rank."""
    uv = _as_edges(uv)
    # n_ids: the id space of the whole graph (as getMaxVid, the same on every rank); the
    # sequence cannot be longer
    cap = max(int(n_ids), int(uv.max()) + 1 if uv.size else 0, 1)
    seq = np.zeros(cap, np.uint32)
    n = ctypes.c_uint32(0)
    rc = capi.lib().sheep_mpi_sequence(_ptr(uv), uv.shape[0], n_ids, mode, _ptr(seq), cap,
                                       ctypes.byref(n))
    if rc == -errno.ERANGE and n.value > 0:
        # some rank's ids do not span the sequence: EVERY rank got -ERANGE with the global
        # length (the smallest buffer of all ranks decides), so every rank retries, including
        # those whose own buffer was large enough (else they would leave the others waiting in
        # the retry's collectives)
        cap = max(cap, n.value)
        seq = np.zeros(cap, np.uint32)
        rc = capi.lib().sheep_mpi_sequence(_ptr(uv), uv.shape[0], n_ids, mode, _ptr(seq), cap,
                                           ctypes.byref(n))
    capi.check(rc, "sheep_mpi_sequence")
    return seq[:n.value]


def build_tree_multi(uv, seq):
    """JTree on this rank's records + mpi_merge: the whole tree, on every rank."""
    uv = _as_edges(uv)
    seq = np.ascontiguousarray(seq, np.uint32)
    n = seq.size
    parent = np.zeros(max(n, 1), np.uint32)
    pst = np.zeros(max(n, 1), np.uint32)
    if n:
        capi.call("sheep_build_tree_multi", _ptr(uv), uv.shape[0], _ptr(seq), n, _ptr(parent),
                  _ptr(pst))
    return JNodeTable(parent[:n], pst[:n])


def partition_edges(uv, parts, seq, n_parts=None):
    """graph2tree -p K -o OUT's edge output (writePartitionedGraph, partition.cpp:588-630) on the
    GPU: a list with, per part, the (X, Y) pairs (X < Y, self-loops skipped) in the writer's
    order (X ascending, then record order)."""
    uv = _as_edges(uv)
    parts = np.ascontiguousarray(parts, np.int16)
    seq = np.ascontiguousarray(seq, np.uint32)
    if n_parts is None:
        n_parts = int(parts.max()) + 1
    out = np.zeros((max(uv.shape[0], 1), 2), np.uint32)
    start = np.zeros(n_parts + 1, np.uint64)
    capi.call("sheep_partition_edges", _ptr(uv), uv.shape[0], _ptr(parts), parts.size, _ptr(seq),
              seq.size, n_parts, _ptr(out), _ptr(start))
    return [out[int(start[p]):int(start[p + 1])] for p in range(n_parts)]
