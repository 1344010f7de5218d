"""The C-ABI library loads (no GPU needed) and exports every symbol include/sheep_amd.h declares."""
import subprocess

from sheep_amd import capi


def test_header_declares_expected_entry_points():
    syms = capi.header_symbols()
    for s in ("sheep_gpu_init", "sheep_degree_seq", "sheep_build_tree", "sheep_merge_trees",
              "sheep_last_error", "sheep_graph2tree_dev", "sheep_merge_trees_dev"):
        assert s in syms


def test_library_exports_every_header_symbol():
    L = capi.lib()
    for s in capi.header_symbols():
        assert hasattr(L, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", capi.lib_path], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(capi.header_symbols()) <= exported


def test_library_is_gfx950_code_object():
    blob = open(capi.lib_path, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the offload bundle's target id


def test_abi_version_and_error_text_without_gpu():
    L = capi.lib()
    assert L.sheep_abi_version() >> 16 == 1
    assert isinstance(L.sheep_last_error(), bytes)


def test_lockstep_entry_points_reject_null_handles_without_gpu():
    """The lockstep calls validate their handle before touching a device (sheep_ls_*)."""
    import ctypes
    import errno

    L = capi.lib()
    for s in ("sheep_ls_begin", "sheep_ls_plan", "sheep_ls_map", "sheep_ls_pack", "sheep_ls_apply",
              "sheep_ls_finish", "sheep_ls_free"):
        assert s in capi.header_symbols()
    n = ctypes.c_uint32(0)
    counts = (ctypes.c_uint64 * 4)()
    assert L.sheep_ls_plan(None, counts, ctypes.byref(n), ctypes.byref(n)) == -errno.EINVAL
    assert b"null" in L.sheep_last_error()
    assert L.sheep_ls_split(None, 0, 2) == -errno.EINVAL
    assert L.sheep_ls_free(None) == 0


def test_host_comm_rejects_bad_arguments_without_gpu():
    """sheep_comm_init_host checks its name and ranks before touching a device or shared
    memory (the multi-process rehearsal's communicator)."""
    import errno

    L = capi.lib()
    assert "sheep_comm_init_host" in capi.header_symbols()
    assert L.sheep_comm_init_host(b"no-slash", 2, 0) == -errno.EINVAL
    assert L.sheep_comm_init_host(b"/sheep-x", 2, 2) == -errno.EINVAL
    assert L.sheep_comm_init_host(None, 2, 0) == -errno.EINVAL


def test_options_read_once_and_settable_without_gpu():
    """Tuning options: defaults from SHEEP_<NAME> once, then only sheep_set_option changes them;
    unknown names are refused."""
    import pytest

    old = capi.set_option("kb_buckets", 7)
    assert capi.set_option("kb_buckets", old) == 7
    for name in ("ls_split", "ls_seq"):  # options added in round 3
        v = capi.set_option(name, 0)
        assert capi.set_option(name, v) == 0
    # removed in round 3, then in round 4 the A/B-only ones (always on now); round 6 the lab mask
    for gone in ("sort", "bin_tm", "bin_scatter", "ep_plain", "seq_compact", "seq_sort",
                 "part_ysort", "kb_refresh", "kb_gbits", "kb_defer", "degb_plain", "degb_hist",
                 "kb_pick", "kb_drop", "lab"):
        with pytest.raises(capi.SheepError):
            capi.set_option(gone, 0)
    with pytest.raises(capi.SheepError):
        capi.set_option("no_such_option", 1)
