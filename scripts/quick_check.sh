#!/bin/bash
# Short GPU-box iteration: GPU tests + timeline + C2/C3 sweep (measurement tool).
# Usage: bash scripts/quick_check.sh TAG [pytest target...]
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-q}; shift; mkdir -p $O
TESTS=${@:-tests -m gpu}
timeout -k 10 400 python -u -m pytest $TESTS -x -q -o addopts="" --timeout 120 --timeout-method thread > $O/qtests_$T.log 2>&1 || { echo "tests failed"; tail -40 $O/qtests_$T.log; exit 3; }
tail -2 $O/qtests_$T.log
timeout -k 10 120 python scripts/rollout_timeline.py c2 > $O/tl_$T.jsonl || exit 4
timeout -k 10 300 python scripts/kernel_sweep.py c2 c3 10000 65536 > $O/sweep_$T.jsonl 2> $O/sweep_$T.err || exit 5
cat $O/tl_$T.jsonl; cat $O/sweep_$T.jsonl
