"""sheep_amd — MI355X build of Sheep's tree-construction hot path.

The product is ``libsheep_amd.so`` (HIP kernels for gfx950 behind the C-ABI declared in
``include/sheep_amd.h``).  This package is the Python view of that ABI:

* :mod:`sheep_amd.capi`     — ctypes bindings; raises :class:`SheepError` on a negative return.
* :mod:`sheep_amd.api`      — the reference's lib/ interface in Python: ``degree_sequence``,
  ``file_sequence``, ``JTree``/``build_tree``, ``JNodeTable.merge``, ``Facts``,
  ``Partition``/``evaluate`` and the .dat/.net/.tre/.seq formats.
* :mod:`sheep_amd.device`   — the device-pointer calls on torch tensors, including the
  multi-GPU driver (``graph2tree_multi``: one process per GPU over the library's own RCCL
  communicator — degree all-reduce, then one kb bucket loop walked by all ranks).
* :mod:`sheep_amd.dist`     — the same multi-rank loop orchestrated from Python over
  torch.distributed (the gloo rehearsal), and the per-rank partial trees merged on rank 0.

There is no CPU fallback: if the HIP library cannot be loaded every compute call raises.
"""
from .capi import SheepError, lib, lib_path  # noqa: F401

__all__ = ["SheepError", "lib", "lib_path"]
