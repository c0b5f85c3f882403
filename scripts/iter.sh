#!/bin/bash
# Short GPU-box iteration: all GPU tests, then the C2 sweep (kernel times + merge phases) and a host-step bench.
# Usage (repo root, on the box): bash scripts/iter.sh TAG
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-it}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -o addopts="" --timeout 120 --timeout-method thread > $O/it_tests_$T.log 2>&1 || { echo "tests failed"; tail -40 $O/it_tests_$T.log; exit 3; }
tail -2 $O/it_tests_$T.log
SWEEP_MODES=quad timeout -k 10 120 python scripts/kernel_sweep.py c2 10000 > $O/it_sweep_$T.jsonl 2> $O/it_sweep_$T.err || { echo "sweep failed"; tail $O/it_sweep_$T.err; exit 4; }
cat $O/it_sweep_$T.jsonl
timeout -k 10 180 python bench.py --steps 2000 --warmup 20 --no-cpu-baseline --extras 0 > $O/it_bench_$T.json 2> $O/it_bench_$T.err || { echo "bench failed"; tail $O/it_bench_$T.err; exit 5; }
cat $O/it_bench_$T.json
