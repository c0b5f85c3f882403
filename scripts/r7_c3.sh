#!/bin/bash
# C3 merge check (GPU box): the CEM / split-merge GPU tests, the merge's phase stamps (probe build), C3 host p50.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-r7c}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_split_merge.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py -m gpu -x -q -o addopts="" --timeout 200 --timeout-method thread > $O/c3_tests_$T.log 2>&1 || { tail -5 $O/c3_tests_$T.log; exit 3; }
tail -1 $O/c3_tests_$T.log
timeout -k 10 200 python scripts/merge_phases.py c3 > $O/merge_phases_c3_$T.json 2> $O/merge_phases_c3_$T.err || { echo phases failed; exit 4; }
cat $O/merge_phases_c3_$T.json
timeout -k 10 300 python scripts/host_ab.py c3 1000 cur=SRBD_NOP=1 > $O/c3_p50_$T.jsonl || exit 5
cat $O/c3_p50_$T.jsonl
