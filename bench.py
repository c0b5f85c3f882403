#!/usr/bin/env python3
"""Benchmark of the MI355X sampling SRBD MPC step (BASELINE.json metric).

metric : "SRBD rollouts/sec + p50 MPC-step ms at N=10k H=12; 1/2/4/8 GPU"
workload (N=1): BASELINE configs[1] = C2, Go2 trot flat, MPPI, N=10 000, H=12, zero-order control.
A step = one full sampling-MPC iteration over one batch of N rollouts: device Philox RNG ->
fused rollout + cost + block softmax partials -> merge (argmin, MPPI update, GRFs, predicted
state) -> warm start of the next step written back on the device.  Inputs are resident in
HBM when the timed region starts; `value` = rollouts of all ranks / max-over-ranks wall time.
`p50_step_ms` / `p99_step_ms` are the host-to-host latency of one `srbd_step` call (state,
reference, contact and parameters in; GRFs, predicted state, parameters out; PCIe included).

N>1 GPUs (torchrun, one rank per GPU): weak scaling, N = 10 000 rows per GPU of ONE MPC problem;
each step ends in one RCCL all-gather of the per-rank partial records (the path's only exchange),
issued by the library on its own stream between the rollout and the merge (torch.distributed only
carries the RCCL unique id and the timing barrier / max-over-ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
if int(os.environ.get("WORLD_SIZE", "1")) > 1 or "--force-sharded" in sys.argv:
    import torch  # noqa: F401  -- before libsrbd_hip.so: one HIP runtime per process (see _lib.py)

from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, Workload, inputs  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
METRIC = "SRBD rollouts/sec + p50 MPC-step ms at N=10k H=12; 1/2/4/8 GPU"


def make_cfg(w: Workload, n_total: int, rank: int, world: int, device: int):
    return _lib.make_config(num_samples=n_total, horizon=w.horizon, method=w.method,
                            parametrization=w.parametrization, num_splines=w.num_splines, mass=w.mass,
                            inertia=w.inertia, dts=np.full(w.horizon, w.dt, np.float32), device_id=device,
                            rank=rank, world_size=world, use_graph=True, sigma_mppi=w.sigma)


def roofline(w: Workload, n_local: int, kern: dict, traffic):
    """Dominant kernel = the rollout launch as the timed chain runs it.

    Algorithmic bytes: each noise row read once and one cost written, N*(4P+4);
    when the launch also draws the next step's noise (fused), + N*4P written.
    Duration: HIP events around each launch on the context stream (kernel_us).  This agrees with
    rocprofv3's kernel-trace average for the same kernel (profiles/).  event_floor_us (the same event
    pair around an empty kernel) is reported beside it for reference and is NOT subtracted: it holds a
    minimal kernel's own duration as well as dispatch.
    """
    P = w.num_params()
    fused = "fused_rollout_us" in kern
    us = kern["fused_rollout_us"] if fused else kern["rollout_us"]
    floor = kern.get("event_floor_us", 0.0)
    algo = n_local * (4 * P + 4) + (n_local * 4 * P if fused else 0)
    achieved = algo / (us * 1e-6) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "kernel": "rollout_quad_kernel" + (" (+ next-step Philox blocks)" if fused else ""),
            "kernel_us": round(us, 3), "event_floor_us": round(floor, 3),
            "algorithmic_bytes_per_launch": algo}


def pmc_traffic(workload_name: str):
    """HBM bytes per rollout launch from the committed rocprofv3 PMC summary, if present."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(workload_name, {}).get("rollout_hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(w: Workload, seconds: float):
    """The C oracle (OpenMP, all host threads offered) on bounded full C2 steps."""
    sys.path.insert(0, ROOT)
    from oracle import c_oracle as co  # test-infrastructure CPU port, used only as this baseline

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    cfg = co.make_cfg(N=w.num_samples, H=w.horizon, method=1 if w.method == "mppi" else 0, param_kind=0,
                      mass=w.mass, inertia=w.inertia, sigma_mppi=w.sigma)
    s, r, c = inputs(w, 0)
    best = np.zeros(w.num_params(), np.float32)
    co.step(cfg, s, r, c, best, seed=42, counter=0, nthreads=threads)  # warm-up
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds and n < 2000:
        best, *_ = co.step(cfg, s, r, c, best, seed=42, counter=n + 1, nthreads=threads)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(w.num_samples * n / dt, 1), "unit": "rollouts/s", "cores": threads, "kind": "port",
            "sample": f"{n} full MPPI steps of C2 (N={w.num_samples}, H={w.horizon}; Philox noise, rollouts, "
                      f"softmax update, GRFs) in {dt:.1f} s, oracle/srbd_oracle.c OpenMP",
            "ms_per_step": round(1e3 * dt / max(n, 1), 3)}


def interface_latency(w: Workload, steps: int):
    """p50 / p99 ms of one MPC step through the reference's Python plugin API at the workload's shape:
    PeriodicGaitGenerator.compute_contact_sequence (C++ host producer) + SRBDControllerInterface.
    compute_control (prepare_state_and_reference, with_newkey, jitted_compute_control, LegsAttr masking),
    dict state in, LegsAttr GRFs out -- the 100 Hz loop's controller cost (srbd_controller_interface.py:113-180)."""
    import copy
    import types

    from quadruped_pympc_amd import config as base
    from quadruped_pympc_amd.config import ROBOTS
    from quadruped_pympc_amd.helpers.periodic_gait_generator import PeriodicGaitGenerator
    from quadruped_pympc_amd.interfaces.srbd_controller_interface import SRBDControllerInterface
    from quadruped_pympc_amd.synthetic import GAITS

    cfg = types.SimpleNamespace(**{k: copy.deepcopy(getattr(base, k)) for k in
                                   ("robot", "mass", "inertia", "hip_height", "gravity_constant", "mpc_params",
                                    "simulation_params")})
    cfg.robot, cfg.mass, cfg.inertia = w.robot, ROBOTS[w.robot][0], np.array(ROBOTS[w.robot][1])
    cfg.mpc_params.update(horizon=w.horizon, sampling_method=w.method, control_parametrization=w.parametrization,
                          num_splines=w.num_splines, num_parallel_computations=w.num_samples, sigma_mppi=w.sigma,
                          grf_max=cfg.mass * 9.81)
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
    assert np.isfinite(np.concatenate([out[0].FL, out[6]])).all()
    iface.controller.close()
    lat = np.array(lat[20:]) * 1e3
    return {"p50_ms": round(float(np.percentile(lat, 50)), 4), "p99_ms": round(float(np.percentile(lat, 99)), 4),
            "steps": steps, "path": "PeriodicGaitGenerator.compute_contact_sequence + "
                                    "SRBDControllerInterface.compute_control (Python plugin API)"}


def tamols_latency(calls: int):
    """p50 / p99 ms of one TAMOLS foothold adaptation for the four legs on stepping_stones_medium (C4):
    13 x 7 patches raycast on the GPU from the device-resident scene + the TAMOLS search, one call
    (srbd_tamols_run_terrain), Go2 trot stance feet."""
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
                               current_feet_pos=feet)
        lat.append(time.perf_counter() - t0)
    srch.close()
    ter.close()
    lat = np.array(lat[10:]) * 1e3
    return {"p50_ms": round(float(np.percentile(lat, 50)), 4), "p99_ms": round(float(np.percentile(lat, 99)), 4),
            "calls": calls, "valid_legs": int(out["valid"].sum()),
            "path": "srbd_tamols_run_terrain: 4 x 13 x 7 raycast patches + TAMOLS, stepping_stones_medium"}


def bench_single(w, args):
    ctx = _lib.Context(make_cfg(w, w.num_samples, 0, 1, 0))
    s, r, c = inputs(w, 0)
    best = np.zeros(ctx.P, np.float32)
    for k in range(max(1, args.warmup)):
        best, _, res, _ = ctx.step(s, r, c, best, seed=42, counter=k)
    # host-to-host latency of one MPC step
    lat = []
    for k in range(args.latency_steps):
        t0 = time.perf_counter()
        best, _, res, _ = ctx.step(s, r, c, best, seed=42, counter=1000 + k)
        lat.append(time.perf_counter() - t0)
    # throughput: K device-resident steps, warm-started on the device
    ctx.bench_device_steps(max(1, args.warmup))
    t0 = time.perf_counter()
    ms_dev = ctx.bench_device_steps(args.steps)
    wall = time.perf_counter() - t0
    kern = ctx.time_kernels(50)
    ctx.close()
    return dict(n_total=w.num_samples, n_local=w.num_samples, wall=wall, ms_dev=ms_dev, lat=lat, kern=kern)


def bench_multi(w, args, rank, world, local_rank):
    import torch
    import torch.distributed as dist

    from quadruped_pympc_amd.sharded import ShardedSamplingMPC

    torch.cuda.set_device(local_rank)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    n_total = w.num_samples * world  # weak scaling: N rows per GPU of one MPC problem
    mpc = ShardedSamplingMPC(make_cfg(w, n_total, rank, world, local_rank), rank, world, local_rank)
    s, r, c = inputs(w, 0)
    best = np.zeros(mpc.P, np.float32)
    for k in range(max(1, args.warmup)):
        best, _, _ = mpc.step(s, r, c, best, seed=42, counter=k)
    lat = []
    for k in range(args.latency_steps):
        dist.barrier()
        t0 = time.perf_counter()
        best, _, _ = mpc.step(s, r, c, best, seed=42, counter=1000 + k)
        lat.append(time.perf_counter() - t0)
    mpc.device_steps(max(1, args.warmup))
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mpc.device_steps(args.steps)  # rollout -> ncclAllGather -> merge per step, driven from C++
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    n_local = mpc.ctx.n_local
    kern = mpc.ctx.time_kernels(20)
    mpc.close()
    dist.destroy_process_group()
    return dict(n_total=n_total, n_local=n_local, wall=wall, ms_dev=None, lat=lat, kern=kern)


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--latency-steps", type=int, default=500)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--extras", type=int, default=200,
                    help="steps of the supplementary interface / TAMOLS latency probes (0: skip)")
    ap.add_argument("--force-sharded", action="store_true", help=argparse.SUPPRESS)  # 1-GPU rehearsal
    args = ap.parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    w = CONFIGS[args.config]
    if world > 1 or args.force_sharded:
        out = bench_multi(w, args, rank, world, local_rank)
    else:
        out = bench_single(w, args)
    if rank != 0:
        return
    lat = np.array(out["lat"]) * 1e3
    ms_per_step = 1e3 * out["wall"] / args.steps
    value = out["n_total"] * args.steps / out["wall"]
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "rollouts/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "p50_step_ms": round(float(np.percentile(lat, 50)), 4),
        "p99_step_ms": round(float(np.percentile(lat, 99)), 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (fixed-seed Go2 state/reference, PGG trot contact sequence, device Philox noise)",
        "config": {"workload": w.name, "num_samples": out["n_total"], "horizon": w.horizon, "method": w.method,
                   "parametrization": w.parametrization, "robot": w.robot, "gait": w.gait,
                   "parallelism": f"rows sharded over {world} GPU(s)" if world > 1 else "single GPU"},
        "kernels_us": {k: round(v, 3) for k, v in out["kern"].items()},
        "roofline": roofline(w, out["n_local"], out["kern"], pmc_traffic(w.name)),
    }
    if out["ms_dev"] is not None:
        line["device_ms_per_step"] = round(out["ms_dev"] / args.steps, 5)
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(w, args.cpu_seconds)
    else:
        line["cpu_baseline"] = None
    if world == 1 and args.extras:  # supplementary latencies of the callers either side of the path
        line["interface_step"] = interface_latency(w, args.extras)
        line["tamols_c4"] = tamols_latency(args.extras)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
