#!/bin/bash
# One GPU-box iteration: the given pytest targets (default: the whole -m gpu suite), then optionally the default
# bench.  Every step runs under its own time limit; the script stops at the first failure or GPU fault.
# Usage (repo root, on the box): bash scripts/gpu_iter.sh TAG [bench|nobench] [pytest args...]
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-it}; B=${2:-nobench}; shift 2; mkdir -p $O
export TMPDIR=/tmp
fault() { grep -q -i -E 'illegal memory access|memory access fault|GPU fault|core dumped|error code 38' "$@"; }
ARGS=${@:-tests -m gpu}
timeout -k 10 900 python -u -m pytest $ARGS -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/tests_$T.log 2>&1
rc=$?; echo "pytest exit=$rc" >> $O/tests_$T.log; tail -4 $O/tests_$T.log
if fault $O/tests_$T.log; then echo "GPU fault in tests"; exit 3; fi
[ $rc -eq 0 ] || exit 4
if [ "$B" = bench ]; then
    timeout -k 10 400 python bench.py > $O/bench_$T.json 2> $O/bench_$T.err; rc=$?
    if fault $O/bench_$T.err; then echo "GPU fault in bench"; exit 3; fi
    [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 $O/bench_$T.err; exit 5; }
    python - $O/bench_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "p50", d["p50_step_ms"], "roofline", d["roofline"]["frac"], d["roofline"]["kernel_us"])
for k in ("north_star_65536", "c3", "c5_1gpu", "c2_rng_jax"):
    if k in d: print(k, d[k]["value"], d[k]["p50_step_ms"], d[k]["kernels_us"])
PY
fi
echo ALLDONE
