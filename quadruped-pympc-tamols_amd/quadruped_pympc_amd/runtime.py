"""Which config and which GPU a zero-argument constructor binds to.

The reference's classes take no arguments and read ``quadruped_pympc.config``
(``srbd_controller_interface.py:4,83``, ``centroidal_nmpc_jax.py:23-33``).  For the one-import swap
to be exact, a constructor called without ``config_module`` here reads that same module when the
reference package is installed, and this package's mirror (``quadruped_pympc_amd.config``) only
when it is not.  A reference package that is installed but fails to import (for example its
``gym_quadruped`` dependency is missing) raises: falling back silently would run the mirror's robot.

Device: ``mpc_params['device_id']`` may be an ordinal or ``'auto'`` (the default when the key is
absent, as in the reference's config).  ``'auto'`` maps replica process i to GPU i mod G
(SURVEY 8(e) replica mode), with i, in order of precedence: ``SRBD_REPLICA_INDEX`` (an explicit
replica index a launcher sets), ``LOCAL_RANK`` under torchrun, the multiprocessing identity of the
process as the last resort (``batched_simulations.py:49-55`` starts one ``Process`` per replica; the
identity also counts Manager / Pool helpers the parent created, so a launcher that creates those should
set ``SRBD_REPLICA_INDEX``), else 0.  It is resolved when the HIP context is created (the first compute
call), never at construction, and the resolution is logged (logger ``quadruped_pympc_amd.runtime``,
INFO) with its source.
"""
from __future__ import annotations

import importlib
import importlib.util
import logging
import multiprocessing
import os

log = logging.getLogger(__name__)

REFERENCE_CONFIG = "quadruped_pympc.config"


def active_config(config_module=None):
    """``config_module`` if given, else the reference's ``quadruped_pympc.config`` when that package is
    importable, else this package's mirror."""
    if config_module is not None:
        return config_module
    try:
        found = importlib.util.find_spec("quadruped_pympc") is not None
    except ValueError:  # a stub in sys.modules without __spec__
        found = True
    if found:
        return importlib.import_module(REFERENCE_CONFIG)
    from . import config as mirror

    return mirror


def replica_source() -> tuple[int, str]:
    """(index, source) of this replica process: SRBD_REPLICA_INDEX, else LOCAL_RANK, else the
    multiprocessing identity (Process-k -> k-1), else (0, 'main')."""
    for var in ("SRBD_REPLICA_INDEX", "LOCAL_RANK"):
        v = os.environ.get(var)
        if v is not None and v.strip().isdigit():
            return int(v), var
    ident = getattr(multiprocessing.current_process(), "_identity", ())
    if ident:
        return ident[0] - 1, "multiprocessing identity"
    return 0, "main"


def replica_index() -> int:
    return replica_source()[0]


def resolve_device_id(spec, device_count=None) -> int:
    """An ordinal from ``spec`` (int, numeric string, None or 'auto')."""
    if spec is None or (isinstance(spec, str) and spec.strip().lower() == "auto"):
        if device_count is None:
            from . import _lib

            device_count = _lib.device_count()
        if device_count < 1:
            return 0  # context creation then fails loudly (no CPU fallback)
        idx, src = replica_source()
        dev = idx % device_count
        log.info("device_id 'auto' -> GPU %d (replica %d from %s, %d GPU(s) visible)", dev, idx, src, device_count)
        return dev
    return int(spec)
