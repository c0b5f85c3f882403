"""ctypes binding of ``libsrbd_hip.so`` (C-ABI declared in ``include/srbd_mpc.h`` and ``include/srbd_host.h``).

The library is the only compute path: there is no CPU fallback.  Loading fails
loudly (ImportError) when the shared object is missing, and creating a context
fails loudly (RuntimeError) when no HIP device is visible.

One HIP runtime per process: the PyTorch-ROCm wheel bundles its own
``libamdhip64.so`` (SONAME ``libamdhip64.so.7``).  A process that uses both this
library and ``torch.cuda`` (the sharded path over RCCL, the GPU tests) must import
torch first; the loader then resolves our ``libamdhip64.so.7`` dependency to
torch's copy.  Loading this library first would leave torch with a second runtime
that finds no GPU.  Set ``SRBD_IMPORT_TORCH=1`` to have this module import torch
before loading the library.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

MAX_HORIZON = 32
MAX_PARAMS = 384
MAX_ELITE = 16

OK, E_INVALID, E_HIP, E_NODEVICE, E_STATE, E_NOMEM = 0, -1, -2, -3, -4, -5
RANDOM_SAMPLING, MPPI, CEM_MPPI = 0, 1, 2
ZERO_ORDER, LINEAR_SPLINE, CUBIC_SPLINE = 0, 1, 2
METHOD_CODES = {"random_sampling": RANDOM_SAMPLING, "mppi": MPPI, "cem_mppi": CEM_MPPI}
PARAM_CODES = {"zero_order": ZERO_ORDER, "linear_spline": LINEAR_SPLINE, "cubic_spline": CUBIC_SPLINE}

_F = C.c_float
_I = C.c_int32
_D = C.c_double
_P = C.c_void_p
_FP = C.POINTER(C.c_float)
_DP = C.POINTER(C.c_double)
_IP = C.POINTER(C.c_int32)


class SrbdConfig(C.Structure):
    _fields_ = [
        ("num_samples", _I), ("horizon", _I), ("method", _I), ("parametrization", _I), ("num_splines", _I),
        ("num_elite", _I), ("device_id", _I), ("rank", _I), ("world_size", _I), ("use_graph", _I),
        ("mass", _F), ("mg", _F), ("grf_min", _F), ("grf_max", _F), ("mu", _F),
        ("inertia", _F * 9), ("dts", _F * MAX_HORIZON), ("q_diag", _F * 24),
        ("sigma_mppi", _F), ("sigma_random_sampling", _F * 3),
    ]


class SrbdResult(C.Structure):
    _fields_ = [("grf", _F * 12), ("predicted_state", _F * 24), ("best_cost", _F), ("best_index", _I),
                ("status", _I), ("best_freq", _F)]


class TamolsParams(C.Structure):
    _fields_ = [
        ("gradient_delta", _D), ("slope_threshold", _D),
        ("w_edge", _D), ("w_rough", _D), ("w_dev", _D), ("w_nominal", _D), ("w_tracking", _D), ("w_stability", _D),
        ("stability_margin", _D), ("swing_time", _D), ("h_des", _D), ("l_min", _D), ("l_max", _D),
        ("box_dx", _D), ("box_dy", _D), ("stance_duration", _D), ("alphas", _D * 5),
    ]


class FootholdIO(C.Structure):
    """srbd_foothold_io (include/srbd_mpc.h): the C4 step's inputs and outputs."""
    _fields_ = [
        ("state_in", _D * 24), ("ref_base", _D * 12), ("seeds", _D * 12), ("hips", _D * 12), ("forward_vel", _D * 3),
        ("current_contact", _D * 4), ("previous_contact", _D * 4), ("yaw", _D), ("dist_x", _D), ("dist_y", _D),
        ("ray_z", _D), ("rows", _I), ("cols", _I),
        ("footholds", _D * 12), ("boxes", _D * 24), ("seed_heights", _D * 4), ("valid", _I * 4),
        ("state_out", _D * 24), ("ref_out", _D * 24), ("scores", _P), ("heightmaps", _P), ("stage", _I), ("pad", _I),
    ]


class InterfaceIO(C.Structure):
    """srbd_interface_io (include/srbd_mpc.h): one SRBDControllerInterface.compute_control step's inputs / outputs."""
    _fields_ = [
        ("state_in", _D * 24), ("ref_in", _D * 24), ("current_contact", _D * 4), ("previous_contact", _D * 4),
        ("sigma_reset", _D), ("key", C.c_uint64 * 2), ("horizon", _I), ("iterations", _I), ("rng", _I), ("cem", _I),
        ("state_out", _D * 24), ("ref_out", _D * 24), ("grf", _D * 12), ("stage", _I), ("pad", _I),
    ]


SIGNATURES = {
    "srbd_num_params": (_I, [C.POINTER(SrbdConfig)]),
    "srbd_device_count": (_I, [_IP]),
    "srbd_abi_version": (_I, []),
    "srbd_create": (_I, [C.POINTER(SrbdConfig), C.POINTER(_P)]),
    "srbd_destroy": (None, [_P]),
    "srbd_last_error": (C.c_char_p, [_P]),
    "srbd_set_stream": (_I, [_P, _P]),
    # host-step pointers are plain addresses (Context passes cached ints: ndarray.ctypes costs ~2.5 us each)
    "srbd_step": (_I, [_P, _P, _P, _P, _I, _P, _P, _P, C.c_uint64, C.c_uint64, C.POINTER(SrbdResult), _P]),
    "srbd_set_gait": (_I, [_P, _FP, _F, _F, _FP, _I, _FP]),
    "srbd_clear_gait": (_I, [_P]),
    "srbd_set_cost_terms": (_I, [_P, _FP, _F, _F]),
    "srbd_set_armed": (_I, [_P, C.c_int32, C.c_uint64]),
    "srbd_armed_stats": (_I, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "srbd_armed_refired": (_I, [_P, C.POINTER(C.c_int64)]),
    "srbd_debug_arm_delay": (_I, [_P, C.c_uint32]),
    "srbd_debug_split_drop": (_I, [_P]),
    "srbd_foothold_chained": (_I, [_P, C.POINTER(C.c_int64)]),
    "srbd_record_floats": (_I, [_P]),
    "srbd_record_floats_host": (_I, [C.POINTER(SrbdConfig)]),
    "srbd_shard_rows": (_I, [C.c_int64, _I, _I, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "srbd_step_local": (_I, [_P, _FP, _FP, _FP, _I, _FP, _FP, _FP, C.c_uint64, C.c_uint64, _P]),
    "srbd_step_finish": (_I, [_P, _P, _I, _FP, _FP, C.POINTER(SrbdResult), _FP]),
    "srbd_finish_host": (_I, [C.POINTER(SrbdConfig), _FP, _I, _FP, _FP, _I, _FP, _FP, C.POINTER(SrbdResult)]),
    "srbd_make_record_host": (_I, [C.POINTER(SrbdConfig), _I, _I, _FP, _FP, _FP]),
    "srbd_bench_device_steps": (_I, [_P, _I, _FP]),
    "srbd_bench_host_steps": (_I, [_P, _FP, _FP, _FP, _I, _I, _FP, _FP, C.c_uint64, C.c_uint64, _I, _FP]),
    "srbd_time_kernels": (_I, [_P, _I, _FP, _FP, _FP, _FP, _FP]),
    "srbd_device_step_local": (_I, [_P, _P]),
    "srbd_device_step_finish": (_I, [_P, _P, _I]),
    "srbd_sync_result": (_I, [_P, _FP, _FP, C.POINTER(SrbdResult)]),
    "srbd_copy_costs": (_I, [_P, _FP]),
    "srbd_get_state": (_I, [_P, _FP, _FP, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "srbd_set_state": (_I, [_P, _FP, _FP, C.c_uint64, C.c_uint64]),
    "srbd_selftest_div": (_I, [_FP, _FP, _I, _FP, _FP]),
    "srbd_selftest_log1p": (_I, [_FP, _I, _FP, _FP, C.POINTER(C.c_int64)]),
    "srbd_debug_merge_phases": (_I, [_P, _I, _FP]),
    "srbd_comm_get_unique_id": (_I, [C.c_char_p, _P]),
    "srbd_comm_init": (_I, [_P, C.c_char_p, _P]),
    "srbd_step_sharded": (_I, [_P, _P, _P, _P, _I, _P, _P, _P, C.c_uint64, C.c_uint64, C.POINTER(SrbdResult), _P]),
    "srbd_sharded_device_steps": (_I, [_P, _I, _FP]),
    "srbd_xgmi_export": (_I, [_P, _P]),
    "srbd_xgmi_connect": (_I, [_P, _P]),
    "srbd_xgmi_connect_local": (_I, [_P, _I]),
    "srbd_xgmi_probe": (_I, [_P, _IP]),
    "srbd_xgmi_disconnect": (_I, [_P]),
    "srbd_tamols_create": (_I, [_I, C.POINTER(_P)]),
    "srbd_tamols_destroy": (None, [_P]),
    "srbd_tamols_last_error": (C.c_char_p, [_P]),
    # TAMOLS array pointers are plain addresses (TamolsSearch passes cached ints; ctypes pointers also work)
    "srbd_tamols_run": (_I, [_P, _P, _I, _I, _P, _P, _P, _P, _P, _P, C.POINTER(TamolsParams), _P, _P, _P, _P, _P]),
}

class SrbdPgg(C.Structure):
    """srbd_pgg (include/srbd_host.h): PeriodicGaitGenerator state."""
    _fields_ = [("duty_factor", _D), ("step_freq", _D), ("phase_signal", _D * 4), ("phase_offset", _D * 4),
                ("init", _I * 4), ("gait_type", _I), ("previous_gait_type", _I), ("horizon", _I)]


SHM_DOUBLES = 75


class ShmMsg(C.Structure):
    """srbd_shm_msg (include/srbd_host.h): one MPC -> WBC message."""
    _fields_ = [("grf", _D * 12), ("footholds", _D * 12), ("joints_pos", _D * 12), ("joints_vel", _D * 12),
                ("joints_acc", _D * 12), ("pred", _D * 12), ("best_freq", _D), ("loop_time", _D), ("stamp", _D)]


class TerrainPrim(C.Structure):
    """srbd_terrain_prim (include/srbd_mpc.h)."""
    _fields_ = [("type", _I), ("pad", _I), ("cx", _D), ("cy", _D), ("cz", _D), ("a", _D), ("b", _D), ("c", _D),
                ("yaw", _D)]


PRIM_BOX, PRIM_CYLINDER = 0, 1
_U64P = C.POINTER(C.c_uint64)
SIGNATURES.update({
    "srbd_pgg_init": (_I, [C.POINTER(SrbdPgg), _I, _D, _D, _I]),
    "srbd_pgg_reset": (_I, [C.POINTER(SrbdPgg)]),
    "srbd_pgg_run": (_I, [C.POINTER(SrbdPgg), _D, _D, _DP]),
    "srbd_pgg_set_phase_signal": (_I, [C.POINTER(SrbdPgg), _DP, _IP]),
    "srbd_pgg_contact_sequence": (_I, [C.POINTER(SrbdPgg), _DP, _IP, _I, _DP, _I]),
    "srbd_prepare_state": (_I, [_DP, _DP, _DP, _DP, _I, _FP, _DP, _DP]),
    "srbd_shm_publish": (_I, [_P, _P, C.POINTER(ShmMsg)]),
    "srbd_shm_read": (_I, [_P, _P, C.POINTER(ShmMsg), _U64P]),
    "srbd_terrain_create": (_I, [_I, C.POINTER(TerrainPrim), _I, _I, _D, _DP, _I, _I, _D, _D, _D, _D, _D,
                                 C.POINTER(_P)]),
    "srbd_terrain_destroy": (None, [_P]),
    "srbd_terrain_last_error": (C.c_char_p, [_P]),
    "srbd_terrain_patches": (_I, [_P, _DP, _DP, _I, _I, _I, _D, _D, _D, _DP]),
    "srbd_tamols_run_terrain": (_I, [_P, _P, _D, _I, _I, _D, _D, _D, _P, _P, _P, _P, _P, _P,
                                     C.POINTER(TamolsParams), _P, _P, _P, _P, _P, _P]),
    "srbd_foothold_mpc_step": (_I, [_P, _P, C.POINTER(TamolsParams), _P, C.POINTER(FootholdIO), _P, _I, _P, _I,
                                    C.c_uint64, C.c_uint64, C.POINTER(SrbdResult)]),
    "srbd_interface_step": (_I, [_P, _P, _P, _P, _I, _P, _I, _P, C.POINTER(SrbdResult)]),
    "srbd_tamols_phases": (_I, [_P, _I, _FP]),
    "srbd_tamols_phases_raw": (_I, [_P, _P]),
    "srbd_set_rng": (_I, [_P, _I]),
    "srbd_get_rng": (_I, [_P]),
    "srbd_draw_noise": (_I, [_P, C.c_uint64, C.c_uint64, _FP]),
    "srbd_time_launch": (_I, [_P, _I, _I, _FP, _IP]),
    "srbd_jax_prng_key": (_I, [C.c_uint64, _P]),
    "srbd_jax_split": (_I, [_P, _I, _I, _P]),
})

# srbd_time_launch kinds (include/srbd_mpc.h)
TL_RNG, TL_ROLLOUT, TL_ROLLOUT_FUSED, TL_STEP_ROLLOUT, TL_STEP_MERGE, TL_EMPTY = range(6)

# device noise streams (include/srbd_mpc.h srbd_set_rng)
RNG_PHILOX, RNG_JAX, RNG_JAX_LEGACY = 0, 1, 2
RNG_CODES = {"philox": RNG_PHILOX, "jax": RNG_JAX, "jax_legacy": RNG_JAX_LEGACY}

LIB_NAME = "libsrbd_hip.so"
LIB_PATH = os.environ.get("SRBD_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)


def _load():
    if os.environ.get("SRBD_IMPORT_TORCH") == "1":
        import torch  # noqa: F401  (one HIP runtime: torch's)
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is not built: run `make -C quadruped-pympc-tamols_amd` (or __graft_entry__.build()). "
            "The sampling MPC has no CPU fallback."
        )
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:  # e.g. a measurement build (probe / ASan variant) made before the ABI grew
            raise ImportError(f"{LIB_PATH} does not export {name}: it is older than include/srbd_mpc.h -- rebuild it "
                              "(make -C quadruped-pympc-tamols_amd [probe|asan], or __graft_entry__.build())") from None
        fn.restype = res
        fn.argtypes = args
    if lib.srbd_abi_version() != 1:
        raise ImportError("libsrbd_hip.so ABI mismatch")
    return lib


lib = _load()


def _load_fast():
    """The CPython glue of the per-MPC-step host path (csrc/srbd_pyfast.c), bound to this library instance; None
    when it is not built (the Python chain then makes the same library calls)."""
    if os.environ.get("SRBD_PYFAST", "1") == "0":
        return None
    try:
        from . import _srbd_fast
    except ImportError:
        return None
    _srbd_fast.bind(*(C.cast(getattr(lib, f), C.c_void_p).value for f in (
        "srbd_interface_step", "srbd_pgg_contact_sequence", "srbd_foothold_mpc_step", "srbd_jax_split")))
    return _srbd_fast


fast = _load_fast()


def fptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(_FP)


def dptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_DP)


def iptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_IP)


def last_error(ctx=None) -> str:
    msg = lib.srbd_last_error(ctx)
    return msg.decode() if msg else ""


def check(rc: int, ctx=None, what: str = "srbd") -> None:
    if rc != OK:
        raise RuntimeError(f"{what} failed ({rc}): {last_error(ctx)}")


def device_count() -> int:
    n = _I(0)
    lib.srbd_device_count(C.byref(n))
    return int(n.value)


def make_config(*, num_samples, horizon, method, parametrization, num_splines=2, num_elite=10, device_id=0, rank=0,
                world_size=1, use_graph=True, mass, inertia, dts, grf_min=0.0, grf_max=None, mu=0.5, q_diag=None,
                sigma_mppi=3.0, sigma_random_sampling=(0.2, 3.0, 10.0)) -> SrbdConfig:
    cfg = SrbdConfig()
    cfg.num_samples = int(num_samples)
    cfg.horizon = int(horizon)
    cfg.method = METHOD_CODES[method] if isinstance(method, str) else int(method)
    cfg.parametrization = PARAM_CODES[parametrization] if isinstance(parametrization, str) else int(parametrization)
    cfg.num_splines = int(num_splines)
    cfg.num_elite = int(num_elite)
    cfg.device_id = int(device_id)
    cfg.rank = int(rank)
    cfg.world_size = int(world_size)
    cfg.use_graph = 1 if use_graph else 0
    cfg.mass = float(np.float32(mass))
    # (self.robot.mass * 9.81) is a Python float, rounded to f32 when divided by the f32 stance count
    cfg.mg = float(np.float32(float(mass) * 9.81))
    cfg.grf_min = float(np.float32(grf_min))
    cfg.grf_max = float(np.float32(grf_max if grf_max is not None else float(mass) * 9.81))
    cfg.mu = float(np.float32(mu))
    inertia = np.asarray(inertia, dtype=np.float32).reshape(9)
    for i in range(9):
        cfg.inertia[i] = float(inertia[i])
    dts = np.asarray(dts, dtype=np.float32).reshape(-1)
    if dts.shape[0] != horizon:
        raise ValueError("dts must have `horizon` entries")
    for i in range(horizon):
        cfg.dts[i] = float(dts[i])
    if q_diag is None:
        q_diag = np.zeros(24, dtype=np.float32)
        q_diag[2] = 1500
        q_diag[3:6] = 200
        q_diag[6:8] = 500
        q_diag[9:11] = 20
        q_diag[11] = 50
    q_diag = np.asarray(q_diag, dtype=np.float32)
    for i in range(24):
        cfg.q_diag[i] = float(q_diag[i])
    cfg.sigma_mppi = float(np.float32(sigma_mppi))
    for i in range(3):
        cfg.sigma_random_sampling[i] = float(np.float32(sigma_random_sampling[i]))
    return cfg


def jax_prng_key(seed: int) -> np.ndarray:
    """srbd_jax_prng_key: jax.random.PRNGKey(seed) as uint32[2] (centroidal_nmpc_jax.py:167)."""
    key = np.zeros(2, np.uint32)
    check(lib.srbd_jax_prng_key(int(seed) & 0xFFFFFFFFFFFFFFFF, key.ctypes.data), None, "srbd_jax_prng_key")
    return key


def jax_split(key, num: int = 2, partitionable: bool = True) -> np.ndarray:
    """srbd_jax_split: jax.random.split(key, num) -> (num, 2) uint32 (with_newkey, centroidal_nmpc_jax.py:498-501)."""
    k = np.ascontiguousarray(np.asarray(key, np.uint32).reshape(2))
    out = np.zeros((int(num), 2), np.uint32)
    check(lib.srbd_jax_split(k.ctypes.data, int(num), 1 if partitionable else 0, out.ctypes.data), None,
          "srbd_jax_split")
    return out


def pack_key(key) -> int:
    """The `seed` argument of srbd_step in a JAX stream mode: key[0] << 32 | key[1]."""
    k = np.asarray(key, np.uint32).reshape(2)
    return (int(k[0]) << 32) | int(k[1])


def num_params(cfg: SrbdConfig) -> int:
    P = lib.srbd_num_params(C.byref(cfg))
    if P < 0:
        raise ValueError("unsupported configuration")
    return P


REC_HDR = 4  # srbd_core.h: [m, s, best row bits, pad]


def node_record_floats(cfg: SrbdConfig) -> int:
    """Floats per node record of the reduction tree (srbd_core.h rec_floats_rank)."""
    K = cfg.num_elite if cfg.method == CEM_MPPI else 1
    P = num_params(cfg)
    return (REC_HDR + P + 2 * K + K * P + 3) // 4 * 4  # padded to 16-byte words (srbd_core.h rec_pad4)


def record_floats_host(cfg: SrbdConfig) -> int:
    """Floats per rank buffer (== srbd_record_floats of a context of this configuration)."""
    n = lib.srbd_record_floats_host(C.byref(cfg))
    if n < 0:
        raise ValueError(f"srbd_record_floats_host failed ({n}): {last_error(None)}")
    return n


def shard_rows(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """(first row, row count) of `rank` of `world`: whole nodes of the reduction tree (srbd_shard_rows)."""
    a, n = C.c_int64(), C.c_int64()
    rc = lib.srbd_shard_rows(int(n_total), int(rank), int(world), C.byref(a), C.byref(n))
    if rc != OK:
        raise ValueError(f"srbd_shard_rows({n_total}, {rank}, {world}) failed ({rc}): {last_error(None)}")
    return a.value, n.value


def make_record_host(cfg: SrbdConfig, rank: int, world: int, costs: np.ndarray, noise_rows: np.ndarray) -> np.ndarray:
    """srbd_make_record_host: one rank's buffer (its exchange-level node records) from its saturated costs and
    noise rows (the rows of shard_rows(N, rank, world))."""
    rec = np.zeros(record_floats_host(_with_shard(cfg, rank, world)), np.float32)
    costs = np.ascontiguousarray(costs, np.float32)
    noise_rows = np.ascontiguousarray(noise_rows, np.float32)
    check(lib.srbd_make_record_host(C.byref(cfg), int(rank), int(world), fptr(costs), fptr(noise_rows), fptr(rec)),
          None, "srbd_make_record_host")
    return rec


def _with_shard(cfg: SrbdConfig, rank: int, world: int) -> SrbdConfig:
    c = SrbdConfig.from_buffer_copy(cfg)
    c.rank, c.world_size = int(rank), int(world)
    return c


def finish_host(cfg: SrbdConfig, records: np.ndarray, state, contact, best, sigma=None, world=None):
    """srbd_finish_host: merge gathered rank buffers (rank order) on the host.  world: the number of buffers
    (default: the world size whose buffers make up `records`)."""
    records = np.ascontiguousarray(records, np.float32)
    if world is None:
        world = next((w for w in range(1, records.size + 1)
                      if w * record_floats_host(_with_shard(cfg, 0, w)) == records.size), None)
        if world is None:
            raise ValueError("records are not a whole number of rank buffers")
    nrec = int(world)
    state = np.ascontiguousarray(state, np.float32).reshape(24)
    contact = np.ascontiguousarray(contact, np.float32)
    best = np.array(best, np.float32).reshape(-1).copy()
    if sigma is not None:
        sigma = np.array(np.broadcast_to(np.asarray(sigma, np.float32), best.shape), np.float32)
    res = SrbdResult()
    check(lib.srbd_finish_host(C.byref(cfg), fptr(records), nrec, fptr(state), fptr(contact), contact.shape[1],
                               fptr(best), fptr(sigma), C.byref(res)), None, "srbd_finish_host")
    return best, sigma, res


class Context:
    """Owns one ``srbd_ctx`` (device buffers, stream, graphs) for one configuration.

    ``step`` copies its inputs into persistent staging arrays whose addresses are cached, so one
    call costs a few numpy copies plus the C call (the MPC step is latency-bound at N = 10 000).
    """

    def __init__(self, cfg: SrbdConfig):
        self.cfg = cfg
        self.P = num_params(cfg)
        self.N = cfg.num_samples
        self.row0, self.n_local = shard_rows(self.N, cfg.rank, max(1, cfg.world_size))
        h = _P()
        rc = lib.srbd_create(C.byref(cfg), C.byref(h))
        if rc != OK:
            raise RuntimeError(f"srbd_create failed ({rc}): {last_error(None)}")
        self.h = h
        self.step_id = 0
        H = cfg.horizon
        self._io = np.zeros(48, dtype=np.float32)  # state | ref
        self._contact = np.zeros((4, H), dtype=np.float32)
        self._best = np.zeros(self.P, dtype=np.float32)
        self._sigma = np.zeros(self.P, dtype=np.float32)
        self._a_state = self._io.ctypes.data
        self._a_ref = self._a_state + 24 * 4
        self._a_contact = self._contact.ctypes.data
        self._a_best = self._best.ctypes.data
        self._a_sigma = self._sigma.ctypes.data

    def close(self):
        if getattr(self, "h", None):
            lib.srbd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc, what):
        check(rc, self.h, what)

    def _stage(self, state, ref, contact, best, sigma, noise):
        io, H = self._io, self.cfg.horizon
        # plain slice stores when the shapes already match (np.reshape's dispatch costs ~1 us a call)
        io[:24] = state if getattr(state, "shape", None) == (24,) else np.reshape(state, 24)
        io[24:] = ref if getattr(ref, "shape", None) == (24,) else np.reshape(ref, 24)
        contact = np.asarray(contact)
        if contact.ndim != 2 or contact.shape[0] != 4 or contact.shape[1] < H:
            raise ValueError("contact_sequence must be (4, >=H)")
        self._contact[...] = contact[:, :H]
        self._best[...] = best if getattr(best, "shape", None) == (self.P,) else np.reshape(best, self.P)
        a_sigma = None
        if sigma is not None:
            self._sigma[...] = np.broadcast_to(np.asarray(sigma, dtype=np.float32), (self.P,))
            a_sigma = self._a_sigma
        a_noise = None
        if noise is not None:
            noise = np.ascontiguousarray(noise, dtype=np.float32)
            if noise.shape != (self.n_local, self.P):
                raise ValueError(f"noise must be ({self.n_local}, {self.P})")
            a_noise = noise.ctypes.data
        return a_sigma, a_noise, noise

    def _call_step(self, fn, name, state, ref, contact, best, sigma, noise, seed, counter, want_costs):
        a_sigma, a_noise, _keep = self._stage(state, ref, contact, best, sigma, noise)
        res = SrbdResult()
        costs = np.empty(self.n_local, dtype=np.float32) if want_costs else None
        rc = fn(self.h, self._a_state, self._a_ref, self._a_contact, self.cfg.horizon, self._a_best, a_sigma, a_noise,
                int(seed), int(counter), C.byref(res), None if costs is None else costs.ctypes.data)
        self.check(rc, name)
        self.step_id += 1
        return self._best.copy(), (self._sigma.copy() if sigma is not None else None), res, costs

    def step(self, state, ref, contact, best, sigma=None, noise=None, seed=42, counter=0, want_costs=False):
        return self._call_step(lib.srbd_step, "srbd_step", state, ref, contact, best, sigma, noise, seed, counter,
                               want_costs)

    def step_sharded(self, state, ref, contact, best, sigma=None, noise_local=None, seed=42, counter=0,
                     want_costs=False):
        """srbd_step_sharded: this rank's rows, the record exchange (xGMI mailboxes or RCCL) and the merge."""
        return self._call_step(lib.srbd_step_sharded, "srbd_step_sharded", state, ref, contact, best, sigma,
                               noise_local, seed, counter, want_costs)

    def copy_costs(self) -> np.ndarray:
        out = np.empty(self.n_local, dtype=np.float32)
        self.check(lib.srbd_copy_costs(self.h, fptr(out)), "srbd_copy_costs")
        return out

    def get_state(self):
        """srbd_get_state: (best, sigma or None, seed, counter) the next device-resident step starts from."""
        best = np.zeros(self.P, np.float32)
        sigma = np.zeros(self.P, np.float32) if self.cfg.method == CEM_MPPI else None
        seed, ctr = C.c_uint64(0), C.c_uint64(0)
        self.check(lib.srbd_get_state(self.h, fptr(best), fptr(sigma), C.byref(seed), C.byref(ctr)), "srbd_get_state")
        return best, sigma, int(seed.value), int(ctr.value)

    def set_state(self, best, sigma, seed: int, counter: int):
        """srbd_set_state: restore a get_state checkpoint for the following device-resident steps."""
        best = np.ascontiguousarray(np.asarray(best, np.float32).reshape(self.P))
        sig = None if sigma is None else np.ascontiguousarray(
            np.broadcast_to(np.asarray(sigma, np.float32), (self.P,)))
        self.check(lib.srbd_set_state(self.h, fptr(best), fptr(sig), int(seed), int(counter)), "srbd_set_state")

    def bench_device_steps(self, steps: int) -> float:
        ms = _F(0)
        self.check(lib.srbd_bench_device_steps(self.h, int(steps), C.byref(ms)), "srbd_bench_device_steps")
        return float(ms.value)

    def bench_host_steps(self, states, refs, contacts, best, sigma=None, seed=42, counter0=0, steps=1000):
        """srbd_bench_host_steps: per-call wall times (us) of `steps` srbd_step calls made from C."""
        st = np.ascontiguousarray(np.asarray(states, np.float32).reshape(-1, 24))
        rf = np.ascontiguousarray(np.asarray(refs, np.float32).reshape(-1, 24))
        ct = np.ascontiguousarray(np.asarray(contacts, np.float32))
        n_in = st.shape[0]
        if ct.ndim != 3 or ct.shape[0] != n_in or ct.shape[1] != 4 or rf.shape[0] != n_in:
            raise ValueError("states / refs (n, 24), contacts (n, 4, >=H)")
        b = np.ascontiguousarray(np.asarray(best, np.float32).reshape(self.P)).copy()
        sg = None if sigma is None else np.ascontiguousarray(np.broadcast_to(np.asarray(sigma, np.float32),
                                                                             (self.P,))).copy()
        lat = np.zeros(int(steps), np.float32)
        self.check(lib.srbd_bench_host_steps(self.h, fptr(st), fptr(rf), fptr(ct), int(ct.shape[2]), n_in, fptr(b),
                                             fptr(sg), int(seed), int(counter0), int(steps), fptr(lat)),
                   "srbd_bench_host_steps")
        self.step_id += 1
        return lat, b, sg

    def time_kernels(self, iters: int):
        r, g, m, f, fl = _F(0), _F(0), _F(0), _F(0), _F(0)
        self.check(lib.srbd_time_kernels(self.h, int(iters), C.byref(r), C.byref(g), C.byref(m), C.byref(f),
                                         C.byref(fl)), "srbd_time_kernels")
        out = {"rollout_us": r.value, "rng_us": g.value, "merge_us": m.value, "event_floor_us": fl.value}
        if f.value > 0:  # rollout launch carrying the next step's draws (what the step chain runs)
            out["fused_rollout_us"] = f.value
        if self.cfg.world_size <= 1:  # the two launches srbd_step issues, exactly as it issues them
            us, form = self.time_launch(TL_STEP_ROLLOUT, iters)
            out["step_rollout_us"] = us
            out["step_rollout_form"] = form
            out["step_merge_us"] = self.time_launch(TL_STEP_MERGE, iters)[0]
        return out

    def time_launch(self, which: int, iters: int = 200):
        """srbd_time_launch: (average us of `iters` back-to-back launches of one kind, form bits)."""
        us, form = _F(0), _I(0)
        self.check(lib.srbd_time_launch(self.h, int(which), int(iters), C.byref(us), C.byref(form)),
                   "srbd_time_launch")
        return float(us.value), int(form.value)

    def merge_phases(self, iters: int = 50):
        """Merge phase durations (us) of block 0; `slice_block`: the same for block 1 of a column-split merge."""
        out = np.zeros(48, np.float32)
        self.check(lib.srbd_debug_merge_phases(self.h, int(iters), fptr(out)), "srbd_debug_merge_phases")

        def one(o):
            d = dict(zip(("min_key", "weighted_sums", "elite", "outputs", "tail", "staged_at", "tail_prep_at",
                          "shader_mhz"), (round(float(x), 3) for x in o[:8])))
            d["marks_us"] = [round(float(x), 3) for x in o[8:24]]  # finer marks from the start (0: unset)
            return d

        d = one(out[:24])
        if out[24:].any():
            d["slice_block"] = one(out[24:])
        return d

    def set_gait(self, timing, pgg_dt: float, duty_factor: float, freq_set, freq_local=None):
        """srbd_set_gait: gait-adaptive sampling for the following steps (see include/srbd_mpc.h)."""
        t = np.ascontiguousarray(np.asarray(timing, np.float32).reshape(4))
        fs = np.ascontiguousarray(np.asarray(freq_set, np.float32).reshape(-1))
        fl = None if freq_local is None else np.ascontiguousarray(np.asarray(freq_local, np.float32).reshape(-1))
        if fl is not None and fl.shape[0] != self.n_local:
            raise ValueError(f"freq_local: {self.n_local} rows expected, got {fl.shape[0]}")
        self.check(lib.srbd_set_gait(self.h, fptr(t), float(pgg_dt), float(duty_factor), fptr(fs), int(fs.shape[0]),
                                     fptr(fl)), "srbd_set_gait")

    def clear_gait(self):
        self.check(lib.srbd_clear_gait(self.h), "srbd_clear_gait")

    def set_cost_terms(self, r_force=(0.0, 0.0, 0.0), w_smooth: float = 0.0, w_cone: float = 0.0):
        """srbd_set_cost_terms: opt-in force regularisation / GRF smoothing / cone-violation terms (all 0: the
        reference's cost)."""
        r = np.ascontiguousarray(np.asarray(r_force, np.float32).reshape(3))
        self.check(lib.srbd_set_cost_terms(self.h, fptr(r), float(w_smooth), float(w_cone)), "srbd_set_cost_terms")

    def set_armed(self, enable: bool = True, deadline_us: int = 0):
        """srbd_set_armed: queue each host step's successor ahead of its input (launch latency off the call;
        outputs unchanged).  deadline_us bounds the armed copy kernel's wait (0: 50 ms)."""
        self.check(lib.srbd_set_armed(self.h, 1 if enable else 0, int(deadline_us)), "srbd_set_armed")

    def armed_stats(self):
        """srbd_armed_stats: (steps served by an armed chain, armed chains cancelled)."""
        a, b = C.c_int64(0), C.c_int64(0)
        self.check(lib.srbd_armed_stats(self.h, C.byref(a), C.byref(b)), "srbd_armed_stats")
        return int(a.value), int(b.value)

    def armed_refired(self) -> int:
        """srbd_armed_refired: claimed chains that had already given up and were re-run unarmed."""
        a = C.c_int64(0)
        self.check(lib.srbd_armed_refired(self.h, C.byref(a)), "srbd_armed_refired")
        return int(a.value)

    def debug_arm_delay(self, delay_us: int):
        """srbd_debug_arm_delay (tests): host sleep between an armed claim and its go word."""
        self.check(lib.srbd_debug_arm_delay(self.h, int(delay_us)), "srbd_debug_arm_delay")

    def debug_split_drop(self):
        """srbd_debug_split_drop (tests): the next column-split merge's hand-off times out (the step fails)."""
        self.check(lib.srbd_debug_split_drop(self.h), "srbd_debug_split_drop")

    def foothold_chained(self) -> int:
        """srbd_foothold_chained: srbd_foothold_mpc_step calls on this context that ran chained on the device."""
        a = C.c_int64(0)
        self.check(lib.srbd_foothold_chained(self.h, C.byref(a)), "srbd_foothold_chained")
        return int(a.value)

    def set_stream(self, stream_handle: int | None):
        """Launch on a caller-owned hipStream_t; None (or 0, the legacy null stream) -> the context's own."""
        self.check(lib.srbd_set_stream(self.h, C.c_void_p(stream_handle) if stream_handle else None), "srbd_set_stream")

    def record_floats(self) -> int:
        return int(lib.srbd_record_floats(self.h))

    def set_rng(self, kind):
        """srbd_set_rng: 'philox' (default), 'jax' (the reference's jax.random stream, partitionable threefry) or
        'jax_legacy' (jax_threefry_partitionable=False).  In the JAX modes `seed` is the packed key (pack_key)."""
        code = RNG_CODES[kind] if isinstance(kind, str) else int(kind)
        self.check(lib.srbd_set_rng(self.h, code), "srbd_set_rng")

    def rng(self) -> int:
        return int(lib.srbd_get_rng(self.h))

    def draw_noise(self, seed: int, counter: int = 0) -> np.ndarray:
        """srbd_draw_noise: the device draws of a step keyed by (seed, counter), (n_local, P) row-major."""
        out = np.zeros((self.n_local, self.P), np.float32)
        self.check(lib.srbd_draw_noise(self.h, int(seed), int(counter), fptr(out)), "srbd_draw_noise")
        return out
