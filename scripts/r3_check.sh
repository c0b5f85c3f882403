#!/bin/bash
# Round-3 GPU-box session: GPU tests, then the default bench and the throughput-shape profiles.
# Usage (repo root, on the box): bash scripts/r3_check.sh TAG [profile configs...]
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-r3}; shift; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/gpu_tests_$T.log 2>&1
rc=$?
echo "pytest exit=$rc" >> $O/gpu_tests_$T.log
tail -3 $O/gpu_tests_$T.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 3;; esac
timeout -k 10 240 python bench.py --steps 2000 --warmup 20 > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed $?"; exit 4; }
bash scripts/r3_profile.sh $T ${@:-ns c3 c5} || exit 5
echo ALLDONE
