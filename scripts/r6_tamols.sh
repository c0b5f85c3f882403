#!/bin/bash
# TAMOLS iteration on the GPU box: the TAMOLS / terrain / C4 parity tests, the TAMOLS probe and the C4 time split.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O; T=${1:-tam}
timeout -k 10 400 python -u -m pytest tests/test_gpu_tamols.py tests/test_tamols_ties.py tests/test_gpu_terrain.py tests/test_gpu_foothold_chain.py tests/test_gpu_c4_pipeline.py -x -q -o addopts="" --timeout 120 --timeout-method thread > $O/tests_$T.log 2>&1 || { echo "tests failed"; tail -40 $O/tests_$T.log; exit 3; }
tail -1 $O/tests_$T.log
timeout -k 10 200 python scripts/tamols_probe.py > $O/tamols_probe_$T.json 2> $O/tamols_probe_$T.err || { echo probe failed; tail -20 $O/tamols_probe_$T.err; exit 4; }
cat $O/tamols_probe_$T.json
timeout -k 10 300 python scripts/c4_split_probe.py > $O/c4_split_$T.json 2> $O/c4_split_$T.err || { echo split failed; tail -20 $O/c4_split_$T.err; exit 5; }
cat $O/c4_split_$T.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_tam_$T -o run --output-format csv -- python3 $R/scripts/tamols_probe.py > /dev/null 2> $O/prof_tam_$T.err || { echo prof failed; exit 6; }
echo DONE
