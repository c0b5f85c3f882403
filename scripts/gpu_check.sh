#!/bin/bash
# One GPU-box session: GPU tests, the default bench, and a rocprofv3 kernel trace of a short bench.
# Usage (from the repo root, on the box): bash scripts/gpu_check.sh TAG
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-run}; mkdir -p $O
timeout -k 10 500 python -m pytest tests -m gpu -q -o addopts="" --timeout 240 -rf > $O/gpu_tests_$T.log 2>&1
echo "pytest exit=$?" >> $O/gpu_tests_$T.log
rc=$(tail -1 $O/gpu_tests_$T.log)
case "$rc" in *"exit=0"|*"exit=1") ;; *) echo "stopping after $rc"; exit 3;; esac
timeout -k 10 300 python scripts/kernel_sweep.py c2 c3 10000 65536 262144 > $O/sweep_$T.jsonl 2> $O/sweep_$T.err || { echo "sweep failed $?"; exit 6; }
timeout -k 10 300 python bench.py --steps 2000 --warmup 20 > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed $?"; exit 4; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 300 --no-cpu-baseline --latency-steps 50 > $O/bench_prof_$T.json 2> $O/bench_prof_$T.err || { echo "rocprof failed $?"; exit 5; }
echo ALLDONE
