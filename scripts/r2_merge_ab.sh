#!/bin/bash
# Merge variants at C2 (MPPI ZO H12, N=10 000): LDS staging on/off, system fence on/off.
# Usage (repo root, on the box): bash scripts/r2_merge_ab.sh TAG
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-ab}; mkdir -p $O
export SWEEP_MODES=quad
timeout -k 10 120 python scripts/kernel_sweep.py c2 10000 > $O/ab_default_$T.jsonl 2>&1 || { echo "default failed $?"; exit 2; }
SRBD_MERGE_FENCE=1 timeout -k 10 120 python scripts/kernel_sweep.py c2 10000 > $O/ab_fence_$T.jsonl 2>&1 || { echo "fence failed $?"; exit 3; }
SRBD_MERGE_STAGE=2 timeout -k 10 120 python scripts/kernel_sweep.py c2 10000 > $O/ab_nostage_$T.jsonl 2>&1 || { echo "nostage failed $?"; exit 4; }
SRBD_MERGE_STAGE=2 SRBD_MERGE_FENCE=1 timeout -k 10 120 python scripts/kernel_sweep.py c2 10000 > $O/ab_old_$T.jsonl 2>&1 || { echo "old failed $?"; exit 5; }
tail -n1 $O/ab_*_$T.jsonl
