"""Armed host steps (srbd_set_armed): the next srbd_step's copy, rollout and merge are queued during the
current one, the copy kernel waiting on a host-mapped word.  The outputs must be those of unarmed steps
bit for bit, on the serve path and on every cancel path (injected noise, a counter jump, another entry
point, the deadline, another context, destroy)."""
import time

import numpy as np
import pytest

from helpers import make_case, product_cfg

pytestmark = pytest.mark.gpu
f32 = np.float32


@pytest.fixture(scope="module")
def lib():
    from quadruped_pympc_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    return _lib


def _inputs(case, k):
    """Step k's state / reference: the case's, nudged so consecutive steps differ."""
    st = case["state"].copy()
    rf = case["ref"].copy()
    st[0:3] += f32(0.001 * k)
    rf[3] += f32(0.01 * (k % 5))
    return st, rf


def _run(lib, case, script, armed, deadline_us=0, stats=None):
    """Run `script` (a list of actions) on a fresh context; returns every step's outputs (and, armed,
    appends (served, cancelled) to `stats`)."""
    ctx = lib.Context(product_cfg(case))
    if armed:
        ctx.set_armed(True, deadline_us)
    best = case["best"].copy()
    sigma = case["sigma"]
    outs = []
    try:
        for k, act in enumerate(script):
            kind = act[0]
            if kind == "step":
                _, ctr, want = act
                st, rf = _inputs(case, k)
                best, sg, res, costs = ctx.step(st, rf, case["contact"], best, sigma=sigma, seed=5, counter=ctr,
                                                want_costs=want)
                if sg is not None:
                    sigma = sg
                outs.append((best.copy(), np.array(res.grf, f32), np.array(res.predicted_state, f32),
                             res.best_cost, res.best_index, costs))
            elif kind == "noise":  # injected perturbations (parity mode)
                st, rf = _inputs(case, k)
                best, sg, res, costs = ctx.step(st, rf, case["contact"], best, sigma=sigma, noise=case["noise"],
                                                seed=5, counter=act[1], want_costs=True)
                outs.append((best.copy(), np.array(res.grf, f32), np.array(res.predicted_state, f32),
                             res.best_cost, res.best_index, costs))
            elif kind == "costs":
                outs.append(("costs", ctx.copy_costs()))
            elif kind == "terms":
                ctx.set_cost_terms(*act[1])
            elif kind == "gait":  # gait-adaptive sampling (device-drawn step frequencies)
                ctx.set_gait(*act[1:])
            elif kind == "sleep":
                time.sleep(act[1])
            elif kind == "state":
                b, s, seed, ctr = ctx.get_state()
                outs.append(("state", b, seed, ctr))
        if stats is not None:
            stats.append(ctx.armed_stats())
    finally:
        ctx.close()
    return outs


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert len(x) == len(y)
        for u, v in zip(x, y):
            if u is None or isinstance(u, str):
                assert u == v
            else:
                np.testing.assert_array_equal(np.asarray(u), np.asarray(v))


@pytest.mark.parametrize("wkey,method,par,N", [
    ("c2", "mppi", "zero_order", 10000),
    ("c2", "random_sampling", "zero_order", 3001),
    ("c3", "cem_mppi", "cubic_spline", 4096),
    ("c2", "mppi", "linear_spline", 65536),
    ("c2", "mppi", "zero_order", 131072),   # unfused draws: the armed chain carries the RNG kernel
    ("c2", "mppi", "zero_order", 65536),    # the rollout launch merges and publishes (final_merge)
    ("c2", "random_sampling", "zero_order", 40000),
    ("c3", "cem_mppi", "cubic_spline", 70000),
])
def test_armed_chain_bitwise(lib, wkey, method, par, N):
    """Consecutive counters: every step after the first is served by the armed chain."""
    case = make_case(wkey, N=N, method=method, par=par)
    script = [("step", 100 + k, k % 7 == 3) for k in range(24)]
    st = []
    _same(_run(lib, case, script, armed=True, stats=st), _run(lib, case, script, armed=False))
    assert st[0] == (23, 0)  # every step but the first was served


def test_armed_cancel_paths(lib):
    case = make_case("c2", N=10000, method="mppi")
    script = ([("step", 10 + k, False) for k in range(4)]
              + [("noise", 50)]                            # injected noise: cancel, parity path
              + [("step", 51, False), ("step", 52, False)]
              + [("step", 90, False)]                      # counter jump
              + [("step", 91, False), ("costs",)]          # another entry point reads the served step's costs
              + [("step", 92, False), ("terms", ((0.1, 0.1, 0.001), 0.01, 5.0)), ("step", 93, False)]
              + [("terms", ((0.0, 0.0, 0.0), 0.0, 0.0)), ("step", 94, False)]
              + [("sleep", 0.03), ("step", 95, False)]     # past half the 20 ms deadline: not served
              + [("step", 96, True), ("state",), ("step", 97, False), ("step", 98, False)])
    st = []
    _same(_run(lib, case, script, armed=True, deadline_us=20000, stats=st), _run(lib, case, script, armed=False))
    # served: 11-13, 52, 91, 96, 98; cancelled by: the noise call, the counter jump, copy_costs, both
    # set_cost_terms, the expired chain before step 95, get_state
    assert st[0] == (7, 7), st


def test_armed_other_context_not_stalled(lib):
    """A second context's call cancels the first's armed step instead of queueing behind its copy kernel
    until the deadline (2 s here); the first context's next step then runs unarmed, same outputs."""
    case = make_case("c2", N=4096, method="mppi")
    a = lib.Context(product_cfg(case))
    b = lib.Context(product_cfg(case))
    ref = lib.Context(product_cfg(case))
    try:
        a.set_armed(True, 2_000_000)
        ba = br = case["best"].copy()
        for k in range(3):
            ba, _, ra, _ = a.step(case["state"], case["ref"], case["contact"], ba, seed=1, counter=k)
            br, _, rr, _ = ref.step(case["state"], case["ref"], case["contact"], br, seed=1, counter=k)
        t0 = time.perf_counter()
        b.step(case["state"], case["ref"], case["contact"], case["best"], seed=9, counter=0)
        assert time.perf_counter() - t0 < 0.5
        ba, _, ra, _ = a.step(case["state"], case["ref"], case["contact"], ba, seed=1, counter=3)
        br, _, rr, _ = ref.step(case["state"], case["ref"], case["contact"], br, seed=1, counter=3)
        np.testing.assert_array_equal(ba, br)
        np.testing.assert_array_equal(np.array(ra.grf), np.array(rr.grf))
        t0 = time.perf_counter()
        a.close()  # armed again after that step: destroy cancels it
        assert time.perf_counter() - t0 < 0.5
    finally:
        a.close()
        b.close()
        ref.close()


def test_armed_deadline_expiry_on_device(lib):
    """The copy kernel gives up at its deadline (5 ms) on its own; the stream drains and the next step
    (not served: past half the deadline) matches the unarmed run."""
    case = make_case("c2", N=2048, method="mppi")
    script = [("step", 0, False), ("step", 1, False), ("sleep", 0.05), ("step", 2, False), ("step", 3, False)]
    st = []
    _same(_run(lib, case, script, armed=True, deadline_us=5000, stats=st), _run(lib, case, script, armed=False))
    assert st[0][0] == 2, st  # steps 1 and 3; step 2 found the chain past its deadline


def test_armed_plugin_api_bitwise(lib):
    """The reference's call path (PeriodicGaitGenerator + SRBDControllerInterface.compute_control, a new
    key per call) with mpc_params['armed_steps']: outputs equal the unarmed loop's bit for bit."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from quadruped_pympc_amd.synthetic import CONFIGS

    runs, st = [], []
    for armed in (True, False):
        outs = []
        bench.interface_latency(CONFIGS["c2"], 12, armed=armed, outputs=outs, stats=st)
        runs.append(outs)
    assert st[0][0] >= 30 and st[1] == (0, 0), st  # 32 calls: all but the first served
    for a, b in zip(*runs):
        assert len(a) == len(b)
        for u, v in zip(a, b):
            if hasattr(u, "FL"):
                for leg in ("FL", "FR", "RL", "RR"):
                    np.testing.assert_array_equal(np.asarray(getattr(u, leg)), np.asarray(getattr(v, leg)))
            elif u is None or isinstance(u, (str, bool)):
                assert u == v
            else:
                np.testing.assert_array_equal(np.asarray(u, dtype=object if isinstance(u, (list, tuple)) else None),
                                              np.asarray(v, dtype=object if isinstance(v, (list, tuple)) else None))


def test_armed_unfused_any_counter(lib):
    """Unfused (N > 65 536): the armed chain draws for whatever (seed, counter) the call brings, so
    counter jumps are served too; outputs equal the unarmed loop's."""
    case = make_case("c2", N=131072, method="mppi")
    script = [("step", c, False) for c in (3, 4, 9, 10, 40, 41, 42, 7)]
    st = []
    _same(_run(lib, case, script, armed=True, stats=st), _run(lib, case, script, armed=False))
    assert st[0] == (7, 0), st


def test_armed_gait_adaptive_bitwise(lib):
    """Gait-adaptive sampling (srbd_set_gait, device-drawn frequencies): armed = unarmed bit for bit,
    set_gait cancels the pending chain, the following steps are served again."""
    case = make_case("c2", N=10000, method="mppi")
    gait = ("gait", (0.1, 0.6, 0.6, 0.1), 0.02, 0.65, np.array((1.4, 2.0, 2.4), f32), None)
    script = ([gait] + [("step", 20 + k, False) for k in range(6)]
              + [("gait", (0.0, 0.5, 0.5, 0.0), 0.02, 0.65, np.array((1.4, 2.0, 2.4), f32), None)]
              + [("step", 26 + k, k == 2) for k in range(5)])
    st = []
    _same(_run(lib, case, script, armed=True, stats=st), _run(lib, case, script, armed=False))
    assert st[0] == (9, 1), st


@pytest.mark.parametrize("N", [10000, 131072, 65536])  # 65 536: the rollout launch publishes the cancel token
def test_claimed_chain_that_gave_up_reruns_unarmed(lib, N):
    """Round-2 advisor finding: a claim younger than half the deadline whose copy kernel has nevertheless
    timed out (the host was delayed between the claim and the go word) must not return the previous
    input's outputs.  The chain then computes nothing and publishes its cancel token; the call re-runs
    unarmed.  Forced here with a 400 us deadline and a 3 ms host delay after each claim (steps timed from
    C: the next call claims well inside half the deadline): every output equals the unarmed loop's bit for
    bit and every claim is counted as re-run."""
    case = make_case("c2", N=N, method="mppi")
    steps = 8
    ref = []
    for armed in (False, True):
        ctx = lib.Context(product_cfg(case))
        states = np.stack([_inputs(case, k)[0] for k in range(steps)])
        refs = np.stack([_inputs(case, k)[1] for k in range(steps)])
        contacts = np.stack([case["contact"]] * steps)
        if armed:
            ctx.set_armed(True, 400)
            ctx.debug_arm_delay(3000)
        lat, best, _ = ctx.bench_host_steps(states, refs, contacts, case["best"], None, 5, 0, steps)
        outs = (best.copy(), ctx.armed_stats(), ctx.armed_refired())
        ctx.close()
        ref.append(outs)
    (b0, _, _), (b1, (served, cancelled), refired) = ref
    np.testing.assert_array_equal(b0, b1)
    assert refired >= 1 and served + refired <= steps, (served, cancelled, refired)
