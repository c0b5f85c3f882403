"""Worker for test_gpu_xgmi.py (run as its own process, tests only).

W ranks as W contexts on the one GPU of the box, mailboxes connected in-process
(srbd_xgmi_connect_local), each rank's blocking call in its own thread (ctypes releases the GIL), so
the W exchange kernels wait for each other exactly as W GPUs do.  A fresh process holds only these
contexts' streams, so each rank's stream gets its own hardware queue (the test starts this worker
with GPU_MAX_HW_QUEUES=16 for the 8-rank case; HIP's default is 4): two ranks' kernels sharing one
queue would serialise and the first would time out waiting for the other.

Prints one JSON object: {case: "ok" | error text}.
"""
import ctypes as C
import json
import os
import sys
import threading
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "quadruped-pympc-tamols_amd"), ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

from helpers import f32, make_case, product_cfg  # noqa: E402
from quadruped_pympc_amd import _lib  # noqa: E402


def run_threads(fns):
    out, errs = [None] * len(fns), []

    def wrap(i, f):
        try:
            out[i] = f()
        except Exception as e:  # surfaced below
            errs.append(repr(e))

    ts = [threading.Thread(target=wrap, args=(i, f)) for i, f in enumerate(fns)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    if errs:
        raise RuntimeError("; ".join(errs))
    return out


def connected(case, W):
    ctxs = [_lib.Context(product_cfg(case, rank=r, world_size=W)) for r in range(W)]
    for cx in ctxs:
        cx.check(_lib.lib.srbd_xgmi_export(cx.h, (C.c_uint8 * 64)()), "srbd_xgmi_export")
    arr = (C.c_void_p * W)(*[cx.h.value for cx in ctxs])
    rc = _lib.lib.srbd_xgmi_connect_local(arr, W)
    assert rc == 0, _lib.last_error(None)
    return ctxs


def probe(cx):
    r = C.c_int32(0)
    cx.check(_lib.lib.srbd_xgmi_probe(cx.h, C.byref(r)), "srbd_xgmi_probe")
    return r.value


def exchange_case(method, W=2, N=4000, ga=False, wkey="c2"):
    case = make_case(wkey, N=N, method=method, seed=23)
    freqs = np.random.default_rng(1).choice(np.array([1.4, 2.0, 2.4], f32), N).astype(f32) if ga else None
    full = _lib.Context(product_cfg(case))
    if ga:
        full.set_gait((0.1, 0.6, 0.6, 0.1), 0.02, 0.65, np.array([1.4, 2.0, 2.4], f32), freqs)
    b0, s0, r0, _ = full.step(case["state"], case["ref"], case["contact"], case["best"], sigma=case["sigma"],
                              noise=case["noise"])
    full.close()
    ctxs = connected(case, W)
    if ga:  # each rank injects the frequencies of its own rows; the best row's travels in the records
        for cx in ctxs:
            cx.set_gait((0.1, 0.6, 0.6, 0.1), 0.02, 0.65, np.array([1.4, 2.0, 2.4], f32),
                        freqs[cx.row0:cx.row0 + cx.n_local])
    oks = run_threads([lambda cx=cx: probe(cx) for cx in ctxs])
    assert all(ok == 1 for ok in oks), f"probe {oks}"

    def host_step(cx):
        rows = case["noise"][cx.row0:cx.row0 + cx.n_local]
        return cx.step_sharded(case["state"], case["ref"], case["contact"], case["best"], sigma=case["sigma"],
                               noise_local=rows)

    for rep in range(2):  # second round: epochs advance, same inputs -> same outputs
        outs = run_threads([lambda cx=cx: host_step(cx) for cx in ctxs])
        for b, sg, res, _ in outs:
            assert res.best_index == r0.best_index, (res.best_index, r0.best_index)
            np.testing.assert_array_equal(b, b0)  # the fixed reduction tree: W-invariant bits
            np.testing.assert_array_equal(np.array(res.grf, f32), np.array(r0.grf, f32))
            if method == "cem_mppi":
                np.testing.assert_array_equal(sg, s0)
            assert res.best_freq == r0.best_freq
        for o in outs[1:]:
            np.testing.assert_array_equal(outs[0][0], o[0])
            np.testing.assert_array_equal(np.array(outs[0][2].grf, f32), np.array(o[2].grf, f32))

    def chain(cx, n):
        ms = C.c_float(0)
        cx.check(_lib.lib.srbd_sharded_device_steps(cx.h, n, C.byref(ms)), "srbd_sharded_device_steps")
        return ms.value

    def synced(cx):
        b = np.zeros(cx.P, f32)
        sg = np.zeros(cx.P, f32)
        res = _lib.SrbdResult()
        cx.check(_lib.lib.srbd_sync_result(cx.h, _lib.fptr(b), _lib.fptr(sg), C.byref(res)), "srbd_sync_result")
        return b, sg, np.array(res.grf, f32), res.best_index

    for n in (6, 7):  # two-step graphs, then the odd tail
        assert all(ms > 0 for ms in run_threads([lambda cx=cx: chain(cx, n) for cx in ctxs]))
        # back-to-back replayed exchanges (one rank may run an exchange ahead of another, the
        # mailbox halves alternate by epoch): every rank ends on bit-identical outputs
        fin = [synced(cx) for cx in ctxs]
        for o in fin[1:]:
            for a, b in zip(fin[0], o):
                np.testing.assert_array_equal(a, b)
    outs = run_threads([lambda cx=cx: host_step(cx) for cx in ctxs])
    for b, _, res, _ in outs:
        assert res.best_index == r0.best_index
        np.testing.assert_array_equal(b, b0)
    for cx in ctxs:
        cx.close()


def bench_case(W=2, N=4000, steps=3):
    """srbd_bench_host_steps on sharded contexts (the bench's timed loop at N > 1 GPUs): every rank ends
    on the same warm start bit for bit, equal to the unsharded loop's (the fixed reduction tree)."""
    case = make_case("c2", N=N, method="mppi", seed=29)
    states = np.stack([case["state"]] * 2)
    refs = np.stack([case["ref"]] * 2)
    contacts = np.stack([case["contact"]] * 2)
    full = _lib.Context(product_cfg(case))
    full.step(case["state"], case["ref"], case["contact"], case["best"], seed=42, counter=0)  # warm up
    lat0, b0, _ = full.bench_host_steps(states, refs, contacts, case["best"], None, 42, 100, steps)
    full.close()
    ctxs = connected(case, W)
    outs = run_threads([lambda cx=cx: cx.bench_host_steps(states, refs, contacts, case["best"], None, 42, 100, steps)
                        for cx in ctxs])
    for lat, b, _ in outs:
        assert lat.shape == (steps,) and (lat > 0).all()
        np.testing.assert_array_equal(b, b0)
    for o in outs[1:]:
        np.testing.assert_array_equal(outs[0][1], o[1])
    for cx in ctxs:
        cx.close()


def timeout_case():
    """A rank whose peer never arrives fails after the bounded wait (2 s) instead of hanging."""
    case = make_case("c2", N=2000, seed=5)
    ctxs = connected(case, 2)
    cx = ctxs[0]  # rank 1 never steps
    rows = case["noise"][cx.row0:cx.row0 + cx.n_local]
    try:
        cx.step_sharded(case["state"], case["ref"], case["contact"], case["best"], noise_local=rows)
    except RuntimeError as e:
        assert "timed out" in str(e), str(e)
    else:
        raise AssertionError("step without its peer did not fail")
    for c in ctxs:
        c.close()


def main():
    res = {}
    cases = [("mppi", lambda: exchange_case("mppi")), ("cem_mppi", lambda: exchange_case("cem_mppi")),
             ("random_sampling", lambda: exchange_case("random_sampling")),
             ("mppi_w3", lambda: exchange_case("mppi", W=3, N=3001)),
             ("mppi_ga_w3", lambda: exchange_case("mppi", W=3, N=3001, ga=True)),
             # C5 (HyQReal bound MPPI, N=524 288) over 8 ranks of 65 536 rows: needs 8 hardware queues
             ("c5_w8", lambda: exchange_case("mppi", W=8, N=524288, wkey="c5")),
             # bench.py's c5_weak line at N = 2: 524 288 rows per rank (thread form, level-1 folds in the launch,
             # rank buffers of 8 level-2 nodes, merge_xchg_kernel)
             ("c5_weak_w2", lambda: exchange_case("mppi", W=2, N=1048576, wkey="c5")), ("bench_w2", bench_case),
             ("timeout", timeout_case)]
    for name, fn in cases:
        try:
            fn()
            res[name] = "ok"
        except Exception:
            res[name] = traceback.format_exc()[-1500:]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
