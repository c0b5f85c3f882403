#!/bin/bash
# One GPU step of a gpurun command: run "$@" under a time limit with output to gpurun_out/$LOG, then stop the
# call (exit 3) on a GPU fault, abort, segfault or timeout -- nothing more runs on the GPU after one.
# Usage: LOG=name.log TMO=seconds bash scripts/gpu_step.sh cmd args...
O=${GRAFT_REPO_ROOT:-.}/gpurun_out; mkdir -p $O
timeout -k 10 ${TMO:-300} "$@" > $O/$LOG 2>&1
rc=$?
tail -4 $O/$LOG
if grep -q -i -E 'illegal memory access|memory access fault|hipErrorLaunchFailure|GPU fault|core dumped' $O/$LOG; then
    echo "GPU fault in $LOG: stopping"; exit 3
fi
case $rc in 0|1) exit 0;; *) echo "rc=$rc in $LOG: stopping"; exit 3;; esac
