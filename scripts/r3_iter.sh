#!/bin/bash
# Round 3 iteration (GPU box): GPU tests, then kernel sweeps (quad) at C2 / north-star / C3.
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
O=gpurun_out; T=${1:-r3h}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest exit=$rc" >> $O/gpu_tests_$T.log; tail -3 $O/gpu_tests_$T.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 3;; esac
SWEEP_MODES=quad timeout -k 10 200 python scripts/kernel_sweep.py c2 10000 65536 > $O/sweep_$T.jsonl 2>&1 || exit 4
SWEEP_MODES=quad timeout -k 10 200 python scripts/kernel_sweep.py c3 65536 >> $O/sweep_$T.jsonl 2>&1 || exit 5
echo ITERDONE
