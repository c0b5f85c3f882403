"""One rank of the cross-process xGMI exchange test (tests/test_gpu_xgmi_xproc.py; tests only).

Usage: xgmi_xproc_worker.py RANK WORLD PORT MODE OUT_JSON

Each rank is its own process with its own HIP runtime (the reference's process model: one controller per
process, simulation/batched_simulations.py:40-58, ros2/run_controller.py:258-362), all on device 0 of the
box.  The 64-byte IPC handles of the ranks' mailboxes travel through a TCP store (rank 0 hosts it), then
every rank runs srbd_xgmi_export -> srbd_xgmi_connect (hipIpcOpenMemHandle of the peers' mailboxes) ->
srbd_xgmi_probe -> srbd_step_sharded, i.e. the cross-process system-scope stores and epoch flags of
merge_xchg_kernel.

MODE "chain": one step on injected noise (rank 0 also runs the unsharded step on the same noise), then 20
steps on device draws with the warm start fed back (rank 0 also runs the unsharded context on the same
keys); every rank writes its per-step best rows and final parameters to OUT_JSON.
MODE "kill": 3 sharded steps, then rank 1 reports idle and sleeps; rank 0 sends it SIGKILL 0.5 s into its
next sharded step (after its record stores, while it waits on rank 1's flag) and records the failure.
"""
import json
import os
import signal
import sys
import threading
import time
import traceback
from datetime import timedelta

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "quadruped-pympc-tamols_amd"), ROOT, os.path.join(ROOT, "tests")]

import ctypes as C  # noqa: E402


def main():
    rank, world, port, mode, out_path = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    from torch.distributed import TCPStore

    store = TCPStore("127.0.0.1", port, world, rank == 0, timeout=timedelta(seconds=60))
    res = {"rank": rank, "pid": os.getpid()}
    try:
        from helpers import make_case, product_cfg
        from quadruped_pympc_amd import _lib

        N = 4000
        case = make_case("c2", N=N, method="mppi", seed=41)
        cx = _lib.Context(product_cfg(case, rank=rank, world_size=world))
        h = (C.c_uint8 * 64)()
        cx.check(_lib.lib.srbd_xgmi_export(cx.h, h), "srbd_xgmi_export")
        store.set(f"handle{rank}", bytes(h))
        store.set(f"pid{rank}", str(os.getpid()))
        handles = b"".join(store.get(f"handle{r}") for r in range(world))
        cx.check(_lib.lib.srbd_xgmi_connect(cx.h, (C.c_uint8 * (64 * world)).from_buffer_copy(handles)),
                 "srbd_xgmi_connect")
        # connect zeroes this rank's epoch flags: no peer may probe (store a flag here) before every rank has
        # connected -- the barrier ShardedSamplingMPC._setup_xgmi gets from its all-reduce
        store.set(f"connected{rank}", "1")
        for r_ in range(world):
            store.get(f"connected{r_}")
        ok = C.c_int32(0)
        cx.check(_lib.lib.srbd_xgmi_probe(cx.h, C.byref(ok)), "srbd_xgmi_probe")
        res["probe"] = ok.value
        store.set(f"probe{rank}", str(ok.value))
        if not all(store.get(f"probe{r}") == b"1" for r in range(world)):
            raise RuntimeError("probe failed on a rank")
        rows = case["noise"][cx.row0:cx.row0 + cx.n_local]
        b, _, r, _ = cx.step_sharded(case["state"], case["ref"], case["contact"], case["best"], noise_local=rows)
        res["inject"] = {"best": b.tolist(), "best_index": int(r.best_index), "grf": list(r.grf)}
        if rank == 0:  # the unsharded step on the same noise
            full = _lib.Context(product_cfg(case))
            b0, _, r0, _ = full.step(case["state"], case["ref"], case["contact"], case["best"], noise=case["noise"])
            res["inject_unsharded"] = {"best": b0.tolist(), "best_index": int(r0.best_index), "grf": list(r0.grf)}
        if mode == "chain":
            best = case["best"].copy()
            res["steps"] = []
            for k in range(20):
                best, _, r, _ = cx.step_sharded(case["state"], case["ref"], case["contact"], best, seed=7, counter=k)
                res["steps"].append(int(r.best_index))
            res["final"] = [float(x).hex() for x in best]
            if rank == 0:
                bu = case["best"].copy()
                res["steps_unsharded"] = []
                for k in range(20):
                    bu, _, ru, _ = full.step(case["state"], case["ref"], case["contact"], bu, seed=7, counter=k)
                    res["steps_unsharded"].append(int(ru.best_index))
                res["final_unsharded"] = bu.tolist()
                full.close()
            store.set(f"done{rank}", "1")
            for r_ in range(world):
                store.get(f"done{r_}")  # no rank closes its mailbox while a peer may still store into it
            cx.close()
        elif mode == "kill":
            best = case["best"].copy()
            for k in range(3):
                best, _, r, _ = cx.step_sharded(case["state"], case["ref"], case["contact"], best, seed=7, counter=k)
            if rank == 1:
                store.set("idle1", "1")
                time.sleep(120)  # killed by rank 0 meanwhile
                return
            store.get("idle1")
            peer = int(store.get("pid1"))
            threading.Timer(0.5, lambda: os.kill(peer, signal.SIGKILL)).start()
            t0 = time.perf_counter()
            try:
                cx.step_sharded(case["state"], case["ref"], case["contact"], best, seed=7, counter=3)
                res["kill"] = "step completed without its peer"
            except RuntimeError as e:
                res["kill"] = str(e)
            res["kill_wait_s"] = time.perf_counter() - t0
            cx.close()
    except Exception:
        res["error"] = traceback.format_exc()[-2000:]
    with open(out_path, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
