#!/bin/bash
# Round-6 iteration on the GPU box: the rollout-form parity tests, then C2 and north-star bench lines.
# Usage: bash scripts/r6_iter.sh TAG [pytest targets...]
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-it}; shift; mkdir -p $O
TESTS=${@:-tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_tree.py tests/test_gpu_step_paths.py}
timeout -k 10 400 python -u -m pytest $TESTS -x -q -o addopts="" --timeout 120 --timeout-method thread > $O/tests_$T.log 2>&1 || { echo "tests failed"; tail -30 $O/tests_$T.log; exit 3; }
tail -2 $O/tests_$T.log
for cfg in c2 ns; do
  timeout -k 10 200 python bench.py --config $cfg --steps 2000 --targets 0 --extras 0 --no-cpu-baseline --other-steps 0 --device-steps 1000 > $O/bench_${T}_$cfg.json 2> $O/bench_${T}_$cfg.err || { echo "bench $cfg failed"; tail -5 $O/bench_${T}_$cfg.err; exit 4; }
  python - "$O/bench_${T}_$cfg.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = d["kernels_us"]
print(d["config"]["workload"], "value", round(d["value"] / 1e6, 1), "M/s p50", d["p50_step_ms"], "dev", d["device_chain"]["ms_per_step"],
      "step_rollout", k.get("step_rollout_us"), "rollout", k.get("rollout_us"), "fused", k.get("fused_rollout_us"), "rng", k.get("rng_us"))
PY
done
echo ALLDONE
