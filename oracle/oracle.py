"""ctypes view of the CPU checker (oracle/sheep_oracle.cpp).  TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg import this.
The product package (``sheep_amd``) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libsheep_oracle.so")
_lib = None

INVALID = 0xFFFFFFFF
LLAMA, FILE = 0, 1

_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
_i16p = np.ctypeslib.ndpointer(np.int16, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        c = ctypes
        sig = {
            "orc_read_dat": (c.c_uint64, [c.c_char_p, c.c_void_p, c.c_uint64]),
            "orc_read_dat_xs1reader": (c.c_uint64, [c.c_char_p, c.c_void_p, c.c_uint64]),
            "orc_read_net": (c.c_uint64, [c.c_char_p, c.c_void_p, c.c_uint64]),
            "orc_degree": (c.c_int64, [_u32p, c.c_uint64, c.c_int, _u32p, c.c_uint32]),
            "orc_sequence": (c.c_uint32, [_u32p, c.c_uint32, _u32p]),
            "orc_build_tree": (c.c_int, [_u32p, c.c_uint64, _u32p, c.c_uint32, _u32p, _u32p]),
            "orc_merge": (c.c_int, [_u32p, _u32p, _u32p, _u32p, c.c_uint32, _u32p, _u32p]),
            "orc_facts": (None, [_u32p, _u32p, c.c_uint32, _u64p]),
            "orc_parttree_new": (c.c_void_p, [_u32p, _u32p, c.c_uint32]),
            "orc_parttree_free": (None, [c.c_void_p]),
            "orc_partition": (c.c_int, [c.c_void_p, _u32p, c.c_uint32, c.c_int, c.c_double,
                                        _i16p, c.c_uint32]),
            "orc_evaluate": (c.c_int, [_u32p, c.c_uint64, _i16p, c.c_uint32, _u32p, c.c_uint32,
                                       _u64p]),
            "orc_time_graph2tree": (c.c_int, [_u32p, c.c_uint64, c.c_uint32,
                                              np.ctypeslib.ndpointer(np.float64)]),
            "orc_time_graph2tree_ir": (c.c_int, [_u32p, c.c_uint64, c.c_uint32, c.c_int,
                                                 np.ctypeslib.ndpointer(np.float64)]),
            "orc_rmat": (None, [c.c_int, c.c_uint64, c.c_uint64, c.c_uint64, _u32p]),
            "orc_powerlaw": (None, [c.c_uint32, c.c_double, c.c_double, c.c_uint64, c.c_uint64,
                                    c.c_uint64, _u32p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _read(fn, path):
    L = lib()
    n = getattr(L, fn)(path.encode(), None, 0)
    if n == 2**64 - 1:
        raise FileNotFoundError(path)
    uv = np.zeros(2 * n, np.uint32)
    getattr(L, fn)(path.encode(), uv.ctypes.data, n)
    return uv.reshape(-1, 2)


def read_dat(path):
    """All 12-byte records (LLAMA's loader)."""
    return _read("orc_read_dat", path)


def read_dat_xs1reader(path):
    """XS1Reader stream: the last record is seen twice (readerwriter.h:50-58)."""
    return _read("orc_read_dat_xs1reader", path)


def read_net(path):
    return _read("orc_read_net", path)


def degree(uv, mode=LLAMA, n_ids=None):
    uv = np.ascontiguousarray(uv, np.uint32)
    if n_ids is None:
        n_ids = int(uv.max()) + 1 if uv.size else 0
    deg = np.zeros(max(n_ids, 1), np.uint32)
    r = lib().orc_degree(uv.reshape(-1), uv.size // 2, mode, deg, n_ids)
    if r < 0:
        raise ValueError("id out of range")
    return deg[:n_ids]


def sequence(deg):
    deg = np.ascontiguousarray(deg, np.uint32)
    seq = np.zeros(max(deg.size, 1), np.uint32)
    n = lib().orc_sequence(deg, deg.size, seq)
    return seq[:n].copy()


def degree_sequence(uv, mode=LLAMA):
    return sequence(degree(uv, mode))


def build_tree(uv, seq):
    uv = np.ascontiguousarray(uv, np.uint32)
    seq = np.ascontiguousarray(seq, np.uint32)
    n = seq.size
    parent = np.zeros(max(n, 1), np.uint32)
    pst = np.zeros(max(n, 1), np.uint32)
    r = lib().orc_build_tree(uv.reshape(-1), uv.size // 2, seq, n, parent, pst)
    if r != 0:
        raise ValueError("orc_build_tree error %d" % r)
    return parent[:n], pst[:n]


def merge(pa, sa, pb, sb):
    n = pa.size
    parent = np.zeros(max(n, 1), np.uint32)
    pst = np.zeros(max(n, 1), np.uint32)
    a = [np.ascontiguousarray(x, np.uint32) for x in (pa, sa, pb, sb)]
    lib().orc_merge(a[0], a[1], a[2], a[3], n, parent, pst)
    return parent[:n], pst[:n]


FACT_KEYS = ("width", "roots", "vheight", "eheight", "verts", "edges", "halo", "core", "fill")


def facts(parent, pst):
    out = np.zeros(9, np.uint64)
    lib().orc_facts(np.ascontiguousarray(parent, np.uint32), np.ascontiguousarray(pst, np.uint32),
                    parent.size, out)
    return dict(zip(FACT_KEYS, (int(x) for x in out)))


class PartTree:
    """A tree opened for partitioning; kids order persists across k like partition_tree."""

    def __init__(self, parent, pst):
        self.h = lib().orc_parttree_new(np.ascontiguousarray(parent, np.uint32),
                                        np.ascontiguousarray(pst, np.uint32), parent.size)

    def partition(self, seq, k, balance=1.03):
        seq = np.ascontiguousarray(seq, np.uint32)
        n_vid = int(seq.max()) + 1
        parts = np.zeros(n_vid, np.int16)
        lib().orc_partition(self.h, seq, seq.size, k, balance, parts, n_vid)
        return parts

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_parttree_free(self.h)
            self.h = None


EVAL_KEYS = ("edges_cut", "vcom_vol", "vertex_bal", "ecv_hash", "hash_bal", "ecv_down",
             "down_bal", "ecv_up", "up_bal", "edges", "nodes")


def evaluate(uv, parts, seq):
    uv = np.ascontiguousarray(uv, np.uint32)
    out = np.zeros(16, np.uint64)
    r = lib().orc_evaluate(uv.reshape(-1), uv.size // 2, np.ascontiguousarray(parts, np.int16),
                           parts.size, np.ascontiguousarray(seq, np.uint32), seq.size, out)
    if r != 0:
        raise ValueError("evaluate: vertex without part")
    return dict(zip(EVAL_KEYS, (int(x) for x in out[:11])))


def powerlaw(n, m, gamma, i0, seed, e_begin=0, e_end=None):
    """Power-law records [e_begin, e_end) (see sheep_amd/csrc/powerlaw.h)."""
    if e_end is None:
        e_end = m
    uv = np.zeros(2 * (e_end - e_begin), np.uint32)
    lib().orc_powerlaw(n, gamma, i0, seed, e_begin, e_end, uv)
    return uv.reshape(-1, 2)


def rmat(scale, edgefactor, seed, e_begin=0, e_end=None):
    m = edgefactor << scale
    if e_end is None:
        e_end = m
    uv = np.zeros(2 * (e_end - e_begin), np.uint32)
    lib().orc_rmat(scale, seed, e_begin, e_end, uv)
    return uv.reshape(-1, 2)


def time_graph2tree(uv, n_ids):
    """(sort_s, map_s, n_seq) of the single-thread CPU restatement, CSR prebuilt (untimed)."""
    uv = np.ascontiguousarray(uv, np.uint32)
    out = np.zeros(3, np.float64)
    lib().orc_time_graph2tree(uv.reshape(-1), uv.size // 2, n_ids, out)
    return float(out[0]), float(out[1]), int(out[2])


def time_graph2tree_ir(uv, n_ids, threads):
    """`mpirun -n threads graph2tree -ir` analogue on threads: (sort_s, map_s, reduce_s, n_seq,
    result equals the serial tree)."""
    uv = np.ascontiguousarray(uv, np.uint32)
    out = np.zeros(5, np.float64)
    lib().orc_time_graph2tree_ir(uv.reshape(-1), uv.size // 2, n_ids, threads, out)
    return out[0], out[1], out[2], int(out[3]), bool(out[4])
