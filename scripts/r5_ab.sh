#!/bin/bash
# Round-5 A/B of the fast tail (GPU box): host-step times (C-timed) with SRBD_FAST_TAIL=0 / 1 for C2 and north-star.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-ab}; mkdir -p $O
for w in c2 ns; do
  timeout -k 10 200 python scripts/host_ab.py $w 2000 slow=SRBD_FAST_TAIL=0 fast=SRBD_FAST_TAIL=1 > $O/ab_${w}_$T.jsonl 2>&1 || { echo "ab $w failed"; tail -5 $O/ab_${w}_$T.jsonl; exit 6; }
  cat $O/ab_${w}_$T.jsonl
done
