#!/bin/bash
# C3 (CEM cubic) iteration on the GPU box: the CEM parity / path tests, then the C3 bench line.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O; T=${1:-c3}
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split_merge.py tests/test_gpu_step_paths.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_interface_step.py tests/test_gpu_sharded.py tests/test_gpu_unfused_steps.py -x -q -o addopts="" --timeout 120 --timeout-method thread > $O/tests_$T.log 2>&1 || { echo "tests failed"; tail -40 $O/tests_$T.log; exit 3; }
tail -1 $O/tests_$T.log
timeout -k 10 200 python bench.py --config c3 --steps 2000 --targets 0 --extras 0 --no-cpu-baseline --other-steps 0 --device-steps 300 > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed"; tail -5 $O/bench_$T.err; exit 4; }
python - "$O/bench_$T.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["config"]["workload"], "value", round(d["value"] / 1e6, 1), "M/s p50", d["p50_step_ms"], "kernels", d["kernels_us"])
PY
echo DONE
