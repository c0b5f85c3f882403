#!/usr/bin/env python3
"""Benchmark of the MI355X sampling SRBD MPC step (BASELINE.json metric).

metric : "SRBD rollouts/sec + p50 MPC-step ms at N=10k H=12; 1/2/4/8 GPU"
workload (N=1 default): BASELINE configs[1] = C2, Go2 trot flat, MPPI, N=10 000, H=12, zero-order.

A step = one host-to-host MPC iteration as the controller interface issues it: state,
reference, contact sequence and warm-start parameters in (a few KB), device Philox noise (the
O(N*P) input is generated and kept in HBM), fused rollout + cost + block softmax partials, merge
(argmin, MPPI/CEM update, GRFs, predicted state), outputs back on the host.  The timed region is
exactly K such steps (`srbd_step` / `srbd_step_sharded`), bracketed by a barrier and a device
synchronisation; `value` = rollouts of all ranks x K / max-over-ranks wall time.  `p50_step_ms` /
`p99_step_ms` are per-step host-to-host latencies (>= 1000 steps).  The timed steps launch their
kernels in the call (as the sharded steps of N > 1 do, so per-N values compare).  One GPU also reports
`armed_step`: the same loop with srbd_set_armed (each srbd_step queues its successor's copy / rollout /
merge behind itself, the copy kernel waiting on a host-mapped word, so the next call stores its inputs
instead of launching; outputs bit-identical); --armed makes that the timed mode.  `device_chain` is the same
step replayed device-resident (warm start kept on the device, hipGraph chain): the bound the host
round trip sits on.

--gpus N > 1 without a torchrun environment: this script starts torchrun itself as a CHILD
process (before torch or the HIP library is loaded), relays rank 0's line and exits with the
child's status.  One rank per GPU; each rank holds its rows of ONE MPC problem; the rank records
are exchanged by the merge kernel over xGMI (IPC-mapped mailboxes; RCCL all-gather fallback).
  --scaling weak   (default for c1-c4): num_samples rows per GPU, N_total = num_samples x N;
  --scaling strong (default for c5)   : N_total = num_samples split over the N GPUs
                                        (C5: 524 288 = 65 536 per GPU at N=8).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
METRIC = "SRBD rollouts/sec + p50 MPC-step ms at N=10k H=12; 1/2/4/8 GPU"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "ns"])
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="multi-GPU: rows per GPU fixed (weak) or total rows fixed (strong); default strong for c5")
    ap.add_argument("--transport", default="auto", choices=["auto", "xgmi", "rccl"])
    ap.add_argument("--latency-steps", type=int, default=1000)
    ap.add_argument("--device-steps", type=int, default=2000, help="steps of the device-resident chain figure")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--armed", action="store_true", help="one GPU: time armed srbd_step calls (srbd_set_armed)")
    ap.add_argument("--other-steps", type=int, default=2000,
                    help="one GPU: steps of the other mode's sample (armed_step / unarmed_step; 0: skip, e.g. under "
                         "rocprofv3 --pmc, whose serialised dispatch makes an armed copy kernel wait out its deadline)")
    ap.add_argument("--targets", type=int, default=1000,
                    help="one GPU, c2: steps of the supplementary north_star_65536 / c3 lines (0: skip)")
    ap.add_argument("--rng", default="philox", choices=["philox", "jax", "jax_legacy"],
                    help="device noise stream of the timed steps (srbd_set_rng): this library's Philox, or the "
                         "reference's jax.random stream (threefry, partitionable / legacy counter layout)")
    ap.add_argument("--sharded", action="store_true",
                    help="run the sharded step (srbd_step_sharded, xGMI exchange) even on one GPU (world 1)")
    ap.add_argument("--num-samples", type=int, default=0, help="override the workload's num_samples")
    ap.add_argument("--extras", type=int, default=200,
                    help="steps of the supplementary interface / TAMOLS latency probes (0: skip)")
    return ap.parse_args(argv)


def torchrun_cmd(gpus: int, argv, port: int, script: str | None = None) -> list:
    """The launcher command of `bench.py --gpus N` without a torchrun environment: one rank per GPU of this node,
    rendezvous on 127.0.0.1, every rank running this script with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), script or os.path.abspath(__file__)] + list(argv)


def spawn_ranks(args, argv, script: str | None = None) -> int:
    """torchrun as a child process (never exec): rank 0's JSON line reaches this process's stdout (the ranks
    inherit it; the others print none) and the child's exit status is returned."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (xGMI mailboxes, RCCL)
    return subprocess.call(torchrun_cmd(args.gpus, argv, port, script), env=env)


# ---------------------------------------------------------------------------------------------- helpers
def host_cores() -> dict:
    """CPUs this process may use: the affinity set, capped by a cgroup CPU quota when one is set."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    usable = min(aff, quota) if quota else aff
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "usable": usable}


def step_inputs(w, count):
    """`count` distinct synthetic steps: state from default_rng(1234 + k), the PGG contact
    sequence advanced 5 sim steps per MPC step."""
    import numpy as np

    from quadruped_pympc_amd.synthetic import contact_sequences, reference, robot_state

    cs = contact_sequences(w.gait, w.horizon, count)
    out = []
    for k in range(count):
        s = robot_state(w.robot, k)
        out.append((s.astype(np.float32), reference(w.robot, s).astype(np.float32), cs[k].astype(np.float32)))
    return out


class KeyChain:
    """The RNG key of step k: Philox (seed 42, counter k), or the reference's jax.random schedule -- the key of
    the interface's first call, with_newkey(PRNGKey(42)), then split(key)[0] per step (NMPC:167, 498-501) --
    packed as srbd_step's seed.  srbd_bench_host_steps advances the key the same way from (at(k), k)."""

    def __init__(self, _lib, rng: str):
        self.lib, self.rng = _lib, rng
        self.keys = []
        if rng != "philox":
            self.part = rng == "jax"
            self.keys.append(_lib.jax_split(_lib.jax_prng_key(42), 2, self.part)[0])

    def at(self, k: int) -> int:
        if self.rng == "philox":
            return 42
        while len(self.keys) <= k:
            self.keys.append(self.lib.jax_split(self.keys[-1], 2, self.part)[0])
        return self.lib.pack_key(self.keys[k])


def make_cfg(_lib, w, n_total: int, rank: int, world: int, device: int):
    import numpy as np

    return _lib.make_config(num_samples=n_total, horizon=w.horizon, method=w.method,
                            parametrization=w.parametrization, num_splines=w.num_splines, mass=w.mass,
                            inertia=w.inertia, dts=np.full(w.horizon, w.dt, np.float32), device_id=device,
                            rank=rank, world_size=world, use_graph=True, sigma_mppi=w.sigma)


def roofline(w, n_local: int, kern: dict, traffic):
    """Dominant kernel = the rollout launch exactly as the timed srbd_step calls issue it (srbd_time_launch
    SRBD_TL_STEP_ROLLOUT: the step input by value (KS), the in-launch final merge (FM) and the next step's
    draws (fused) where they apply), so the rocprofv3 row of the same instantiation agrees (profiles/).

    achieved = ALGORITHMIC bytes (each noise row read once + one cost written, 4P+4 per
    rollout, x the rows one launch processes) / the launch's average duration (one hipEvent pair on the
    context stream around back-to-back launches).  The fused next-step draws (N*4P stored) are work the
    launch also does but not algorithmic bytes of the rollout: reported as launch_bytes beside it.
    traffic = HBM bytes per launch of that instantiation from the rocprofv3 PMC passes (FETCH_SIZE x2 +
    WRITE_SIZE, profiles/pmc_traffic.json).
    """
    P = w.num_params()
    if "step_rollout_us" in kern:
        form = int(kern.get("step_rollout_form", 0))
        us = kern["step_rollout_us"]
    else:  # sharded contexts: the rollout launch of the step (+ draws when fused)
        form = 1 if kern.get("fused_rollout_us", 0.0) > 0 else 0
        us = kern["fused_rollout_us"] if form else kern["rollout_us"]
    fused = bool(form & 1)
    algo = n_local * (4 * P + 4)
    achieved = algo / (us * 1e-6) / 1e9
    tags = [t for b, t in ((2, "step input by value (KS)"), (4, "in-launch final merge (FM)"),
                           (1, "+ next-step draw blocks"), (16, "one-count fast tail"),
                           (32, "the step's draws made in the launch, no RNG launch")) if form & b]
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "kernel": ("rollout_kernel" if form & 8 else "rollout_quad_kernel") + " as srbd_step launches it"
                      + (" (" + ", ".join(tags) + ")" if tags else ""),
            "kernel_us": round(us, 3), "algorithmic_bytes_per_launch": algo,
            "launch_bytes": algo + (n_local * 4 * P if fused else 0), "bytes_per_rollout": 4 * P + 4}


def pmc_traffic(workload_name: str):
    """HBM bytes per rollout launch from the committed rocprofv3 PMC summary, if present."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(workload_name, {}).get("rollout_hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def supplementary(_lib, key: str, steps: int, rng: str = "philox"):
    """A shape beside the headline line (one GPU): BASELINE north_star's MPPI ZO N=65 536 H=12 ("ns"), C3 (CEM
    cubic N=65 536 H=16), C5's 524 288 rows on one GPU (the denominator of the strong-scaling ratio), or C2 on
    another noise stream.  Host-to-host srbd_step latencies timed from C, the device-resident chain,
    per-kernel averages and the rollout roofline, measured as for the headline."""
    import numpy as np

    from quadruped_pympc_amd.synthetic import CONFIGS

    w = CONFIGS[key]
    ctx = _lib.Context(make_cfg(_lib, w, w.num_samples, 0, 1, 0))
    if rng != "philox":
        ctx.set_rng(rng)
    keys = KeyChain(_lib, rng)
    ins = step_inputs(w, 32)
    best = np.zeros(ctx.P, np.float32)
    sigma = np.full(ctx.P, 3.0, np.float32) if w.method == "cem_mppi" else None
    arrs = (np.stack([x[0] for x in ins]), np.stack([x[1] for x in ins]), np.stack([x[2] for x in ins]))
    _, best, sigma = ctx.bench_host_steps(*arrs, best, sigma, keys.at(0), 0, 20)  # warm-up
    t_us, best, sigma = ctx.bench_host_steps(*arrs, best, sigma, keys.at(20), 20, steps)
    ctx.bench_device_steps(20)
    ms = ctx.bench_device_steps(steps)
    kern = ctx.time_kernels(200)
    ctx.close()
    return {"workload": w.name, "num_samples": w.num_samples, "horizon": w.horizon, "method": w.method,
            "parametrization": w.parametrization, "rng": rng,
            "value": round(w.num_samples / (float(t_us.mean()) * 1e-6), 1), "unit": "rollouts/s",
            "ms_per_step": round(float(t_us.mean()) * 1e-3, 5),
            "p50_step_ms": round(float(np.percentile(t_us, 50)) * 1e-3, 4),
            "p99_step_ms": round(float(np.percentile(t_us, 99)) * 1e-3, 4), "steps": int(t_us.size),
            "device_chain": {"value": round(w.num_samples * steps / (ms * 1e-3), 1),
                             "ms_per_step": round(ms / steps, 5), "steps": steps},
            "kernels_us": {k: round(v, 3) for k, v in kern.items()},
            # form bit 32: the step's draws are made inside its rollout launch (rng_us times the RNG launch the step
            # no longer issues)
            "step_draws": "in the rollout launch" if int(kern.get("step_rollout_form", 0)) & 32 else "RNG launch or fused",
            "roofline": roofline(w, w.num_samples, kern, pmc_traffic(w.name))}


def cpu_baseline(w, seconds: float):
    """The C port of the step (oracle/srbd_oracle.c, OpenMP over samples) on every usable host core, on
    a bounded sample of full steps of the same workload (the JAX-CPU reference cannot run: JAX absent)."""
    import numpy as np

    sys.path.insert(0, ROOT)
    from oracle import c_oracle as co  # test-infrastructure CPU port, used only as this baseline

    cores = host_cores()
    threads = cores["usable"]
    method = {"random_sampling": 0, "mppi": 1, "cem_mppi": 2}[w.method]
    kind = {"zero_order": 0, "linear_spline": 1, "cubic_spline": 2}[w.parametrization]
    cfg = co.make_cfg(N=w.num_samples, H=w.horizon, method=method, param_kind=kind, num_splines=w.num_splines,
                      mass=w.mass, inertia=w.inertia, sigma_mppi=w.sigma)
    ins = step_inputs(w, 8)
    P = co.num_params(cfg)
    best = np.zeros(P, np.float32)
    sigma = np.full(P, 3.0, np.float32) if w.method == "cem_mppi" else None
    s, r, c = ins[0]
    co.step(cfg, s, r, c, best, sigma=sigma, seed=42, counter=0, nthreads=threads)  # warm-up
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds and n < 2000:
        s, r, c = ins[n % len(ins)]
        best, sig, *_ = co.step(cfg, s, r, c, best, sigma=sigma, seed=42, counter=n + 1, nthreads=threads)
        sigma = sig if sigma is not None else None
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(w.num_samples * n / dt, 1), "unit": "rollouts/s", "cores": threads, "kind": "port",
            "nproc": cores["nproc"], "affinity_cpus": cores["affinity"], "cgroup_quota_cpus": cores["cgroup_quota_cpus"],
            "sample": f"{n} full {w.method} steps of {w.name} (N={w.num_samples}, H={w.horizon}; Philox noise, "
                      f"rollouts, update, GRFs) in {dt:.1f} s, oracle/srbd_oracle.c OpenMP on {threads} threads "
                      f"(all usable host CPUs: affinity {cores['affinity']}, nproc {cores['nproc']})",
            "ms_per_step": round(1e3 * dt / max(n, 1), 3)}


def interface_latency(w, steps: int, armed: bool = False, outputs: list | None = None, stats: list | None = None):
    """p50 / p99 ms of one MPC step through the reference's Python plugin API at the workload's shape:
    PeriodicGaitGenerator.compute_contact_sequence (C++ host producer) + SRBDControllerInterface.
    compute_control (prepare_state_and_reference, with_newkey, jitted_compute_control, LegsAttr masking),
    dict state in, LegsAttr GRFs out -- the 100 Hz loop's controller cost (srbd_controller_interface.py:113-180)."""
    import copy
    import types

    import numpy as np

    from quadruped_pympc_amd import config as base
    from quadruped_pympc_amd.config import ROBOTS
    from quadruped_pympc_amd.helpers.periodic_gait_generator import PeriodicGaitGenerator
    from quadruped_pympc_amd.interfaces.srbd_controller_interface import SRBDControllerInterface
    from quadruped_pympc_amd.synthetic import GAITS, inputs

    cfg = types.SimpleNamespace(**{k: copy.deepcopy(getattr(base, k)) for k in
                                   ("robot", "mass", "inertia", "hip_height", "gravity_constant", "mpc_params",
                                    "simulation_params")})
    cfg.robot, cfg.mass, cfg.inertia = w.robot, ROBOTS[w.robot][0], np.array(ROBOTS[w.robot][1])
    cfg.mpc_params.update(horizon=w.horizon, sampling_method=w.method, control_parametrization=w.parametrization,
                          num_splines=w.num_splines, num_parallel_computations=w.num_samples, sigma_mppi=w.sigma,
                          grf_max=cfg.mass * 9.81, device_id=0, armed_steps=armed)
    iface = SRBDControllerInterface(cfg)
    gtype, freq, duty = GAITS[w.gait]
    pgg = PeriodicGaitGenerator(duty, freq, gtype, w.horizon)
    s, r, _ = inputs(w, 0)
    legs = ("FL", "FR", "RL", "RR")
    state = {"position": s[0:3], "linear_velocity": s[3:6], "orientation": s[6:9], "angular_velocity": s[9:12]}
    state.update({"foot_" + n: s[12 + 3 * i:15 + 3 * i] for i, n in enumerate(legs)})
    ref = {"ref_position": r[0:3], "ref_linear_velocity": r[3:6], "ref_orientation": r[6:9],
           "ref_angular_velocity": r[9:12]}
    ref.update({"ref_foot_" + n: r[12 + 3 * i:15 + 3 * i].reshape(1, 3) for i, n in enumerate(legs)})
    dts, lens = np.array([w.dt]), np.array([w.horizon])
    lat = []
    for k in range(steps + 20):
        for _ in range(5):
            pgg.run(0.002, pgg.step_freq)
        t0 = time.perf_counter()
        cs = pgg.compute_contact_sequence(dts, lens)
        out = iface.compute_control(state, ref, cs, cfg.inertia, pgg.phase_signal, pgg.step_freq, 0)
        lat.append(time.perf_counter() - t0)
        if outputs is not None:
            outputs.append(out)
    assert np.isfinite(np.concatenate([out[0].FL, out[6]])).all()
    if stats is not None:
        stats.append(iface.controller.context.armed_stats())
    iface.controller.close()
    lat = np.array(lat[20:]) * 1e3
    return {"p50_ms": round(float(np.percentile(lat, 50)), 4), "p99_ms": round(float(np.percentile(lat, 99)), 4),
            "steps": steps, "path": "PeriodicGaitGenerator.compute_contact_sequence + "
                                    "SRBDControllerInterface.compute_control (Python plugin API)"
                                    + (", mpc_params['armed_steps']" if armed else "")}


def tamols_latency(calls: int):
    """p50 / p99 ms of one TAMOLS foothold adaptation for the four legs on stepping_stones_medium (C4):
    13 x 7 patches raycast on the GPU from the device-resident scene + the TAMOLS search, one call
    (srbd_tamols_run_terrain), Go2 trot stance feet."""
    import numpy as np

    from quadruped_pympc_amd import config
    from quadruped_pympc_amd.helpers.terrain import GpuTerrain
    from quadruped_pympc_amd.helpers.visual_foothold_adaptation import TamolsSearch, tamols_params_struct

    ter = GpuTerrain.stepping_stones()
    srch = TamolsSearch(0)
    params = dict(config.simulation_params["tamols_params"])
    params["h_des"] = 0.25
    ps = tamols_params_struct(params, "go2")
    feet = np.array([[1.22, 0.13, 0.05], [1.22, -0.13, 0.05], [0.84, 0.13, 0.05], [0.84, -0.13, 0.05]])
    hips = feet + np.array([0.0, 0.0, 0.3])
    contact = np.array([0, 1, 1, 0], np.int32)
    lat = []
    for k in range(calls + 10):
        seeds = feet + np.array([0.12 + 0.001 * (k % 7), 0.01, 0.0])
        t0 = time.perf_counter()
        out = srch.run_terrain(ter, 0.0, seeds, hips, ps, forward_vel=np.array([0.5, 0.0, 0.0]),
                               base_position=np.array([1.03, 0.0, 0.35]), current_contact=contact,
                               current_feet_pos=feet, want_scores=False, want_heightmaps=False)
        lat.append(time.perf_counter() - t0)
    srch.close()
    ter.close()
    lat = np.array(lat[10:]) * 1e3
    return {"p50_ms": round(float(np.percentile(lat, 50)), 4), "p99_ms": round(float(np.percentile(lat, 99)), 4),
            "calls": calls, "valid_legs": int(out["valid"].sum()),
            "path": "srbd_tamols_run_terrain: 4 x 13 x 7 raycast patches + TAMOLS, stepping_stones_medium",
            "cadence": "every call adapts (the reference adapts at the swing apex only, wb_interface.py:230-246)"}


def c4_pipeline_latency(steps: int):
    """C4 as one per-MPC-step sequence (BASELINE configs[3]; helpers/foothold_pipeline.py): the four heightmap
    patches raycast on the GPU from the device-resident stepping_stones_medium scene and TAMOLS in one launch, the
    adapted footholds into ref_state, SRBDControllerInterface.compute_control (prepare_state_and_reference + the
    MPPI N = 10 000 H = 12 step on device draws; one host call, srbd_foothold_mpc_step, when the config allows) --
    timed around the whole step from Python."""
    import numpy as np

    from quadruped_pympc_amd.helpers.foothold_pipeline import TamolsMpcStep
    from quadruped_pympc_amd.helpers.legs_attr import LegsAttr
    from quadruped_pympc_amd.helpers.terrain import GpuTerrain
    from quadruped_pympc_amd.synthetic import CONFIGS, c4_config, c4_inputs

    w = CONFIGS["c4"]
    ter = GpuTerrain.stepping_stones()
    pipe = TamolsMpcStep(ter, c4_config())
    ins = [c4_inputs(k) for k in range(16)]
    lat = []
    for k in range(steps + 20):
        state, seeds, hips, ref_base, cs = ins[k % len(ins)]
        t0 = time.perf_counter()
        out = pipe.step(state, LegsAttr(*seeds), LegsAttr(*hips), ref_base, cs, state["linear_velocity"],
                        state["orientation"], state["angular_velocity"], np.zeros(4), 1.4)
        lat.append(time.perf_counter() - t0)
    assert np.isfinite(out[6]).all()
    valid = sum(pipe.last_constraints[n] is not None for n in ("FL", "FR", "RL", "RR"))
    fused = pipe._fusable()
    chained = pipe.controller.context.foothold_chained()
    pipe.close()
    ter.close()
    lat = np.array(lat[20:])
    return {"value": round(w.num_samples / float(lat.mean()), 1), "unit": "rollouts/s",
            "p50_ms": round(float(np.percentile(lat, 50)) * 1e3, 4),
            "p99_ms": round(float(np.percentile(lat, 99)) * 1e3, 4), "steps": steps, "valid_legs": int(valid),
            "workload": w.name, "fused": bool(fused), "chained_steps": int(chained),
            "cadence": "TAMOLS runs on every MPC step here; the reference adapts only at the swing apex "
                       "(wb_interface.py:230-246), so this is an upper bound on its per-step cost",
            "path": "TamolsMpcStep.step: GpuHeightMap x4 (lazy) -> VisualFootholdAdaptation.compute_adaptation "
                    "(srbd_tamols_run_terrain: raycast + TAMOLS, one launch) -> ref_state -> "
                    "SRBDControllerInterface.compute_control (srbd_prepare_state, srbd_step MPPI N=10000 H=12); "
                    "fused: one host call, srbd_foothold_mpc_step -- chained on the device (the TAMOLS launch writes "
                    "the step's input, the rollout launch queued behind it, one host wait) when the context allows"}


# ---------------------------------------------------------------------------------------------- runs
def run_steps(step_fn, ins, best, first_counter, count, lat=None):
    """`count` host-to-host steps, counters consecutive (the fused next-step draws are used)."""
    for i in range(count):
        s, r, c = ins[(first_counter + i) % len(ins)]
        t0 = time.perf_counter()
        best = step_fn(s, r, c, best, first_counter + i)
        if lat is not None:
            lat.append(time.perf_counter() - t0)
    return best


def bench_single(_lib, w, args):
    import numpy as np

    ctx = _lib.Context(make_cfg(_lib, w, w.num_samples, 0, 1, 0))
    if args.rng != "philox":
        ctx.set_rng(args.rng)
    keys = KeyChain(_lib, args.rng)
    ins = step_inputs(w, 32)
    best = np.zeros(ctx.P, np.float32)
    sigma = np.full(ctx.P, 3.0, np.float32) if w.method == "cem_mppi" else None
    state = {"sigma": sigma}

    def step(s, r, c, b, k):
        b, sg, _, _ = ctx.step(s, r, c, b, sigma=state["sigma"], seed=keys.at(k), counter=k)
        if sg is not None:
            state["sigma"] = sg
        return b

    armed = bool(args.armed)
    ctx.set_armed(armed, 0)
    k = 0
    best = run_steps(step, ins, best, k, max(1, args.warmup))
    k += max(1, args.warmup)
    # the timed steps: srbd_step called from C (srbd_bench_host_steps), each call host-to-host at the
    # C-ABI boundary (returns with GRFs / prediction / parameters on the host)
    states = np.stack([x[0] for x in ins])
    refs = np.stack([x[1] for x in ins])
    contacts = np.stack([x[2] for x in ins])
    lat = []
    if args.steps < args.latency_steps:  # latency sample of >= latency_steps steps besides the timed region
        l_us, best, state["sigma"] = ctx.bench_host_steps(states, refs, contacts, best, state["sigma"], keys.at(k), k,
                                                          args.latency_steps)
        lat = list(l_us * 1e-6)
        k += args.latency_steps
    # W more untimed steps in the same C loop right before the timed ones (the Python-driven warmup above ran
    # before the latency sample)
    _, best, state["sigma"] = ctx.bench_host_steps(states, refs, contacts, best, state["sigma"], keys.at(k), k,
                                                   max(1, args.warmup))
    k += max(1, args.warmup)
    t0 = time.perf_counter()
    t_us, best, state["sigma"] = ctx.bench_host_steps(states, refs, contacts, best, state["sigma"], keys.at(k), k,
                                                      args.steps)
    wall = time.perf_counter() - t0
    k += args.steps
    if not lat:
        lat = list(t_us * 1e-6)
    # the other mode over a sample of the same loop
    other = None
    if args.other_steps > 0:
        ctx.set_armed(not armed, 0)
        n_other = max(200, min(args.steps, args.other_steps))
        o_us, best, state["sigma"] = ctx.bench_host_steps(states, refs, contacts, best, state["sigma"], keys.at(k), k,
                                                          n_other)
        k += n_other
        o_us = o_us[min(20, n_other // 10):]
        other = {"value": round(w.num_samples / (float(o_us.mean()) * 1e-6), 1),
                 "ms_per_step": round(float(o_us.mean()) * 1e-3, 5),
                 "p50_step_ms": round(float(np.percentile(o_us, 50)) * 1e-3, 4),
                 "p99_step_ms": round(float(np.percentile(o_us, 99)) * 1e-3, 4), "steps": int(o_us.size)}
    served, cancelled = ctx.armed_stats()
    ctx.set_armed(False, 0)
    # the same steps through the Python ctypes wrapper (Context.step), for the binding's overhead
    py = []
    best = run_steps(step, ins, best, k, min(300, max(20, args.latency_steps // 4)), py)
    dev = None
    if args.device_steps > 0:
        ctx.bench_device_steps(max(1, args.warmup))
        ms = ctx.bench_device_steps(args.device_steps)
        dev = {"value": round(w.num_samples * args.device_steps / (ms * 1e-3), 1),
               "ms_per_step": round(ms / args.device_steps, 5), "steps": args.device_steps}
    kern = ctx.time_kernels(200)
    ctx.close()
    return dict(n_total=w.num_samples, n_local=w.num_samples, wall=wall, lat=lat, kern=kern, dev=dev,
                transport=None, py_lat=py, armed=armed, other=other, arm_stats=(served, cancelled),
                timed_us=[round(float(x), 2) for x in t_us] if args.steps <= 64 else None)


def bench_multi(_lib, w, args, rank, world, local_rank, scaling, steps=None, device_steps=None):
    """One sharded workload on this rank's GPU (the process group is up); steps / device_steps override args."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from quadruped_pympc_amd.sharded import ShardedSamplingMPC

    steps = args.steps if steps is None else steps
    device_steps = args.device_steps if device_steps is None else device_steps
    n_total = w.num_samples if scaling == "strong" else w.num_samples * world
    mpc = ShardedSamplingMPC(make_cfg(_lib, w, n_total, rank, world, local_rank), rank, world, local_rank,
                             transport=args.transport, rng=args.rng)
    keys = KeyChain(_lib, args.rng)
    ins = step_inputs(w, 32)
    best = np.zeros(mpc.P, np.float32)
    sigma = np.full(mpc.P, 3.0, np.float32) if w.method == "cem_mppi" else None
    state = {"sigma": sigma}

    def step(s, r, c, b, k):
        b, sg, _ = mpc.step(s, r, c, b, sigma=state["sigma"], seed=keys.at(k), counter=k)
        if sg is not None:
            state["sigma"] = sg
        return b

    k = 0
    best = run_steps(step, ins, best, k, max(1, args.warmup))
    k += max(1, args.warmup)
    lat = []
    if steps < args.latency_steps:
        dist.barrier()
        best = run_steps(step, ins, best, k, args.latency_steps, lat)
        k += args.latency_steps
    # library-owned exchange (xGMI mailboxes / RCCL): the steps are timed from C like the one-GPU path
    c_timed = mpc.transport in ("xgmi", "rccl")
    arrs = (np.stack([x[0] for x in ins]), np.stack([x[1] for x in ins]), np.stack([x[2] for x in ins]))
    dist.barrier()
    torch.cuda.synchronize()
    timed = []
    t0 = time.perf_counter()
    if c_timed:  # rollout -> xGMI record exchange -> merge, srbd_step_sharded from C
        t_us, best, state["sigma"] = mpc.ctx.bench_host_steps(*arrs, best, state["sigma"], keys.at(k), k, steps)
        timed = list(t_us * 1e-6)
    else:
        best = run_steps(step, ins, best, k, steps, timed)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dist.barrier()
    t = torch.tensor([wall], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    if not lat:
        lat = timed
    dev = None
    if device_steps > 0:
        mpc.device_steps(max(1, args.warmup))
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mpc.device_steps(device_steps)
        torch.cuda.synchronize()
        dwall = time.perf_counter() - t0
        t = torch.tensor([dwall], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dwall = float(t.item())
        dev = {"value": round(n_total * device_steps / dwall, 1),
               "ms_per_step": round(1e3 * dwall / device_steps, 5), "steps": device_steps}
    n_local = mpc.ctx.n_local
    kern = mpc.ctx.time_kernels(100)
    transport = mpc.transport
    transports = [None] * world  # the exchange every rank set up (xgmi, or rccl after a failed probe)
    dist.all_gather_object(transports, transport)
    mpc.close()
    return dict(n_total=n_total, n_local=n_local, wall=wall, lat=lat, kern=kern, dev=dev, transport=transport,
                transports=transports, steps=steps, world=world)


def rows_per_rank(n_total: int, world: int):
    """Every rank's row count under the fixed reduction tree's partition (srbd_shard_rows; ADVICE r4: balance)."""
    from quadruped_pympc_amd import _lib

    return [_lib.shard_rows(n_total, r, world)[1] for r in range(world)]


def multi_line(w, out, scaling):
    """The per-workload summary of a sharded run (the supplementary C5 lines at N > 1)."""
    import numpy as np

    lat = np.array(out["lat"]) * 1e3
    return {"value": round(out["n_total"] * out["steps"] / out["wall"], 1), "unit": "rollouts/s",
            "scaling": scaling, "num_samples": out["n_total"], "rows_per_gpu": out["n_local"],
            "rows_per_rank": rows_per_rank(out["n_total"], out.get("world", 1)),
            "ms_per_step": round(1e3 * out["wall"] / out["steps"], 5), "steps": out["steps"],
            "p50_step_ms": round(float(np.percentile(lat, 50)), 4), "transport": out["transport"],
            "transport_per_rank": out.get("transports"),
            "kernels_us": {k: round(v, 3) for k, v in out["kern"].items()}}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args, argv))  # before torch / the HIP library are loaded
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # exactly one line on stdout: native libraries (RCCL's version banner at communicator setup, ...) print to fd 1, so
    # fd 1 is pointed at stderr for the run and the JSON line goes to the saved stdout
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
    if world > 1 or args.sharded:
        import torch  # noqa: F401  -- before libsrbd_hip.so: one HIP runtime per process (see _lib.py)
    import numpy as np

    from quadruped_pympc_amd import _lib
    from quadruped_pympc_amd.synthetic import CONFIGS

    w = CONFIGS[args.config]
    if args.num_samples > 0:
        import dataclasses

        w = dataclasses.replace(w, num_samples=args.num_samples, name=f"{w.name}_n{args.num_samples}")
    scaling = args.scaling or ("strong" if args.config == "c5" else "weak")
    extra = {}
    if world > 1 or args.sharded:
        if "WORLD_SIZE" not in os.environ:  # --sharded on one GPU without a launcher: a group of one
            with socket.socket() as s_:
                s_.bind(("127.0.0.1", 0))
                os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s_.getsockname()[1]), RANK="0",
                                  WORLD_SIZE="1", LOCAL_RANK="0")
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        out = bench_multi(_lib, w, args, rank, world, local_rank, scaling)
        if world > 1 and args.targets > 0 and args.config == "c2":
            # BASELINE configs[4] beside the headline: C5's 524 288 rows split over the N GPUs (strong; the
            # one-GPU line's c5_1gpu is its denominator) and 524 288 rows per GPU (weak)
            c5 = CONFIGS["c5"]
            for sc in ("strong", "weak"):
                o = bench_multi(_lib, c5, args, rank, world, local_rank, sc, steps=args.targets, device_steps=0)
                extra[f"c5_{sc}"] = multi_line(c5, o, sc)
        dist.destroy_process_group()
    else:
        out = bench_single(_lib, w, args)
    if rank != 0:
        return
    single = world == 1 and not args.sharded
    lat = np.array(out["lat"]) * 1e3
    line = {
        "metric": METRIC,
        "value": round(out["n_total"] * args.steps / out["wall"], 1),
        "unit": "rollouts/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * out["wall"] / args.steps, 5),
        "p50_step_ms": round(float(np.percentile(lat, 50)), 4),
        "p99_step_ms": round(float(np.percentile(lat, 99)), 4),
        "latency_steps": int(lat.size),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (fixed-seed robot states / references, PGG contact sequences, device "
                + ("Philox noise" if args.rng == "philox" else "jax.random (threefry) noise") + ")",
        "rng": args.rng,
        "config": {"workload": w.name, "num_samples": out["n_total"], "rows_per_gpu": out["n_local"],
                   "rows_per_rank": rows_per_rank(out["n_total"], world),
                   **({"transport_per_rank": out["transports"]} if out.get("transports") else {}),
                   "horizon": w.horizon, "method": w.method, "parametrization": w.parametrization,
                   "robot": w.robot, "gait": w.gait,
                   "parallelism": (f"rows sharded over {world} GPUs ({scaling} scaling), record exchange: "
                                   f"{out['transport']}") if not single else "single GPU"},
        "step": (("armed " if out.get("armed") else "")
                 + "host-to-host srbd_step, timed around each call in C (srbd_bench_host_steps; state/ref/contact/"
                 "params in, GRFs/pred/params out; noise device-resident)") if single else
                (f"host-to-host srbd_step_sharded ({out['transport']} record exchange), "
                 + ("timed in C (srbd_bench_host_steps)" if out["transport"] in ("xgmi", "rccl")
                    else "through the Python binding") + ", max over ranks"),
        "device_chain": out["dev"],
        **({("unarmed_step" if out["armed"] else "armed_step"): out["other"],
            "armed_served_cancelled": list(out["arm_stats"])} if single else {}),
        "python_step": ({"p50_ms": round(float(np.percentile(np.array(out["py_lat"]) * 1e3, 50)), 4),
                         "steps": len(out["py_lat"]), "path": "Context.step (ctypes) -> srbd_step"}
                        if out.get("py_lat") else None),
        "kernels_us": {k: round(v, 3) for k, v in out["kern"].items()},
        **({"timed_step_us": out["timed_us"]} if out.get("timed_us") else {}),
        "roofline": roofline(w, out["n_local"], out["kern"], pmc_traffic(w.name)),
        **extra,
    }
    if single and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(w, args.cpu_seconds)
    else:
        line["cpu_baseline"] = None
    if single and args.targets > 0 and args.config == "c2":  # the north-star shape, C3 and C5 beside the headline
        line["north_star_65536"] = supplementary(_lib, "ns", args.targets, args.rng)
        line["c3"] = supplementary(_lib, "c3", args.targets, args.rng)
        # C5's 524 288 rows on one GPU: the denominator of the driver's C5 strong-scaling ratio
        line["c5_1gpu"] = supplementary(_lib, "c5", args.targets, args.rng)
        # every shape on the other noise stream too (Philox <-> the reference's jax.random stream, which the
        # drop-in Sampling_MPC draws by default)
        other = "jax" if args.rng == "philox" else "philox"
        line["c2_rng_" + other] = supplementary(_lib, "c2", args.targets, other)
        line["north_star_65536_rng_" + other] = supplementary(_lib, "ns", args.targets, other)
        line["c3_rng_" + other] = supplementary(_lib, "c3", args.targets, other)
        line["c5_1gpu_rng_" + other] = supplementary(_lib, "c5", args.targets, other)
    if single and args.extras and args.config in ("c2", "c4"):  # the callers either side of the path
        line["interface_step"] = interface_latency(w, args.extras)
        line["interface_step_armed"] = interface_latency(w, args.extras, armed=True)
        line["tamols_c4"] = tamols_latency(args.extras)
        line["c4"] = c4_pipeline_latency(args.extras)
    sys.stdout.flush()
    buf = (json.dumps(line) + "\n").encode()
    while buf:
        buf = buf[os.write(out_fd, buf):]


if __name__ == "__main__":
    main()
    # teardown marker: a run that printed this and then did not exit hung in process teardown
    print("bench: body done", file=sys.stderr, flush=True)
