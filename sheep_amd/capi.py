"""ctypes bindings for libsheep_amd.so (include/sheep_amd.h).

Host-pointer calls take numpy arrays; device-pointer calls take integer device addresses
(e.g. ``tensor.data_ptr()`` of a torch tensor on ``cuda``) and an optional HIP stream handle.
"""
import ctypes
import errno
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
lib_path = os.path.join(_HERE, "libsheep_amd.so")
header_path = os.path.join(_ROOT, "include", "sheep_amd.h")

DEGREE_LLAMA = 0
DEGREE_FILE = 1
INVALID = 0xFFFFFFFF


class SheepError(RuntimeError):
    """A negative return from the C-ABI; ``.code`` is the (negative) errno."""

    def __init__(self, code, msg):
        super().__init__("%s (%s)" % (msg, errno.errorcode.get(-code, code)))
        self.code = code


_lib = None


def build():
    """Compile the HIP library in-tree (hipcc --offload-arch=gfx950)."""
    import subprocess

    subprocess.run(["make", "-s", "-C", os.path.join(_HERE, "csrc")], check=True)


def header_symbols():
    """Every function the public header declares."""
    text = open(header_path).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sheep_\w+)\s*\(", text, re.M)))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(lib_path):
        raise SheepError(-errno.ENOENT, "libsheep_amd.so not built: run sheep_amd.capi.build()")
    L = ctypes.CDLL(lib_path)
    c = ctypes
    u32p, vp = c.c_void_p, c.c_void_p
    sigs = {
        "sheep_gpu_init": [c.c_int],
        "sheep_release": [],
        "sheep_abi_version": [],
        "sheep_last_error": [],
        "sheep_degree_seq": [u32p, c.c_uint64, c.c_uint32, c.c_int, u32p, u32p, u32p],
        "sheep_build_tree": [u32p, c.c_uint64, u32p, c.c_uint32, u32p, u32p],
        "sheep_merge_trees": [u32p, u32p, u32p, u32p, c.c_uint32, u32p, u32p],
        "sheep_degree_dev": [u32p, c.c_uint64, c.c_uint32, c.c_int, u32p, vp],
        "sheep_degree_ex_dev": [u32p, c.c_uint64, c.c_uint32, c.c_int, u32p, u32p, vp],
        "sheep_sequence_dev": [u32p, c.c_uint32, u32p, u32p, u32p, vp],
        "sheep_build_tree_deg_dev": [u32p, c.c_uint64, u32p, c.c_uint32, u32p, c.c_uint32, u32p,
                                     u32p, c.c_int, u32p, u32p, vp],
        "sheep_build_tree_dev": [u32p, c.c_uint64, u32p, c.c_uint32, c.c_uint32, u32p, u32p, vp],
        "sheep_merge_trees_dev": [u32p, u32p, u32p, u32p, c.c_uint32, vp],
        "sheep_merge_forests_dev": [u32p, c.c_uint32, c.c_uint32, u32p, vp],
        "sheep_evaluate_dev": [u32p, c.c_uint64, vp, u32p, c.c_uint32, c.c_uint32, vp, vp],
        "sheep_evaluate": [u32p, c.c_uint64, vp, c.c_uint32, u32p, c.c_uint32, c.c_uint32, vp],
        "sheep_graph2tree_dev": [u32p, c.c_uint64, c.c_uint32, c.c_int, u32p, u32p, u32p, u32p,
                                 vp],
        "sheep_rmat_dev": [u32p, c.c_int, c.c_uint64, c.c_uint64, c.c_uint64, vp],
        "sheep_powerlaw_dev": [u32p, c.c_uint32, c.c_double, c.c_double, c.c_uint64, c.c_uint64,
                               c.c_uint64, vp],
        "sheep_last_timings": [c.c_void_p, c.c_void_p, c.c_int],
        "sheep_ls_begin": [u32p, c.c_uint64, u32p, c.c_uint32, u32p, c.c_uint32, u32p, vp, vp,
                           vp, vp],
        "sheep_ls_plan": [vp, vp, vp, vp],
        "sheep_ls_split": [vp, c.c_uint32, c.c_uint32],
        "sheep_ls_map": [vp, c.c_uint32, vp, vp, vp, vp],
        "sheep_ls_pack": [vp, c.c_uint32, vp, c.c_uint32, vp],
        "sheep_ls_apply": [vp, c.c_uint32, vp, c.c_uint32, c.c_uint32, vp],
        "sheep_ls_finish": [vp, u32p, u32p, u32p, c.c_int, u32p, u32p, vp],
        "sheep_ls_free": [vp],
        "sheep_comm_unique_id": [vp],
        "sheep_comm_init": [vp, c.c_int, c.c_int],
        "sheep_comm_init_host": [c.c_char_p, c.c_int, c.c_int],
        "sheep_comm_free": [],
        "sheep_comm_info": [vp, vp],
        "sheep_mpi_sequence": [u32p, c.c_uint64, c.c_uint32, c.c_int, u32p, c.c_uint32, u32p],
        "sheep_build_tree_multi": [u32p, c.c_uint64, u32p, c.c_uint32, u32p, u32p],
        "sheep_mpi_merge": [u32p, u32p, c.c_uint32],
        "sheep_partition_edges_dev": [u32p, c.c_uint64, vp, u32p, c.c_uint32, c.c_uint32, u32p, vp,
                                      vp],
        "sheep_partition_edges": [u32p, c.c_uint64, vp, c.c_uint32, u32p, c.c_uint32, c.c_uint32,
                                  u32p, vp],
        "sheep_graph2tree_multi_dev": [u32p, c.c_uint64, c.c_uint32, c.c_int, u32p, u32p, u32p,
                                       u32p, vp],
        "sheep_graph2tree_multi_local": [vp, vp, c.c_uint32, c.c_uint32, c.c_int, u32p, u32p, u32p,
                                         u32p],
        "sheep_set_option": [c.c_char_p, c.c_longlong],
        "sheep_records_register": [u32p, c.c_uint64],
        "sheep_records_release": [u32p],
        "sheep_records_load_dat": [c.c_char_p, c.c_uint64, c.c_uint64, u32p, c.c_uint64, vp, vp],
        "sheep_read_dat_dev": [c.c_char_p, c.c_uint64, c.c_uint64, u32p, c.c_uint64, vp, vp, vp],
        "sheep_get_option": [c.c_char_p, c.c_void_p],
        "sheep_partition": [u32p, u32p, c.c_uint32, u32p, vp, c.c_uint32, c.c_double, vp,
                            c.c_uint32, vp],
    }
    for name, args in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = c.c_char_p if name == "sheep_last_error" else c.c_int
    _lib = L
    return L


def check(r, name):
    """Raise SheepError for a negative ABI return r of function `name`."""
    if r < 0:
        raise SheepError(r, "%s: %s" % (name, lib().sheep_last_error().decode()))
    return r


def call(name, *args):
    """Invoke an ABI function; raise SheepError on a negative return."""
    return check(getattr(lib(), name)(*args), name)


def last_timings():
    L = lib()
    names = (ctypes.c_char_p * 32)()
    ms = (ctypes.c_double * 32)()
    n = L.sheep_last_timings(names, ms, 32)
    return [(names[i].decode(), ms[i]) for i in range(n)]


def set_option(name, value):
    """sheep_set_option: a tuning option (results never depend on it); returns the old value."""
    old = ctypes.c_longlong(0)
    call("sheep_get_option", name.encode(), ctypes.byref(old))
    call("sheep_set_option", name.encode(), int(value))
    return old.value
