"""C4 per-MPC-step latency (bench.c4_pipeline_latency) with srbd_foothold_mpc_step chained on the device and as
the sequence of calls (SRBD_FOOTHOLD_CHAIN=0), alternating runs; one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
import bench  # noqa: E402
out = {}
for rep in range(2):
    for mode in ("1", "0"):
        os.environ["SRBD_FOOTHOLD_CHAIN"] = mode
        r = bench.c4_pipeline_latency(2000)
        out.setdefault("chain" if mode == "1" else "sequential", []).append(
            {k: r[k] for k in ("p50_ms", "p99_ms", "chained_steps")})
print(json.dumps(out))
