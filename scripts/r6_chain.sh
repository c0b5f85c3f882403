#!/bin/bash
# C4 chained foothold step on the GPU box: the parity tests, the time split, a kernel trace of chained steps.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O; T=${1:-chain}
timeout -k 10 400 python -u -m pytest tests/test_gpu_foothold_chain.py tests/test_gpu_c4_pipeline.py -x -q -o addopts="" --timeout 120 --timeout-method thread > $O/tests_$T.log 2>&1 || { echo "tests failed"; tail -40 $O/tests_$T.log; exit 3; }
tail -1 $O/tests_$T.log
timeout -k 10 300 python scripts/c4_split_probe.py > $O/c4_split_$T.json 2> $O/c4_split_$T.err || { echo probe failed; tail -20 $O/c4_split_$T.err; exit 4; }
cat $O/c4_split_$T.json
cd /tmp && export TMPDIR=/tmp
SRBD_FOOTHOLD_CHAIN=1 timeout -k 10 180 rocprofv3 --kernel-trace -d $O/trace_$T -o run --output-format csv -- python3 $R/scripts/c4_split_probe.py 300 > $O/c4_split_trace_$T.json 2> $O/c4_split_trace_$T.err || { echo trace failed; tail -5 $O/c4_split_trace_$T.err; exit 5; }
echo DONE
