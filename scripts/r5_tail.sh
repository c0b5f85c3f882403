#!/bin/bash
# Round-5 tail iteration (GPU box): the step-path / tree / split-merge parity tests, the step-tail stamps (probe
# build) for C2 and north-star, then a short C2 + north-star bench.  Each step under its own limit; stops at the
# first failure.  Usage: bash scripts/r5_tail.sh TAG
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-t}; mkdir -p $O
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_gpu_step_paths.py tests/test_gpu_tree.py tests/test_gpu_split_merge.py tests/test_gpu_fullsize.py}
timeout -k 10 600 python -u -m pytest $TESTS \
    -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/tail_tests_$T.log 2>&1
rc=$?; tail -3 $O/tail_tests_$T.log; [ $rc -eq 0 ] || exit 3
for w in c2 ns; do
  timeout -k 10 120 python scripts/step_tail.py $w > $O/tail_${w}_$T.json 2> $O/tail_${w}_$T.err || { echo "step_tail $w failed"; exit 4; }
  cat $O/tail_${w}_$T.json
done
timeout -k 10 300 python bench.py --steps 2000 --no-cpu-baseline --other-steps 1000 > $O/bench_$T.json 2> $O/bench_$T.err || { echo bench failed; tail -5 $O/bench_$T.err; exit 5; }
python - $O/bench_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "p50", d.get("p50_step_ms"), "roofline", d["roofline"]["frac"], d["roofline"].get("kernel_us"))
for k in ("north_star_65536", "c3", "c5_1gpu", "c2_rng_jax"):
    if k in d: print(k, d[k]["value"], d[k].get("p50_step_ms"), d[k].get("kernels_us"))
PY
echo ALLDONE
