#!/bin/bash
# TAMOLS check on the GPU box: the TAMOLS / terrain / C4 GPU tests, the kernel under rocprofv3 (tamols_probe.py: phase
# stamps + host p50), the chained C4 step split (c4_split_probe.py).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-r7t}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tamols.py tests/test_gpu_terrain.py tests/test_gpu_foothold_chain.py tests/test_gpu_c4_pipeline.py tests/test_tamols_ties.py -m gpu -x -q -o addopts="" --timeout 120 --timeout-method thread > $O/tamols_tests_$T.log 2>&1 || { tail -5 $O/tamols_tests_$T.log; exit 3; }
tail -1 $O/tamols_tests_$T.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_c4_$T -o run --output-format csv -- python3 $R/scripts/tamols_probe.py > $O/tamols_probe_$T.json 2> $O/tamols_probe_$T.err || { echo tamols prof failed; exit 4; }
cat $O/tamols_probe_$T.json
grep tamols $O/prof_c4_$T/*kernel_stats.csv | cut -c1-60,150-
timeout -k 10 300 python scripts/c4_split_probe.py > $O/c4_split_$T.json 2> $O/c4_split_$T.err || { echo c4 split failed; exit 5; }
cat $O/c4_split_$T.json
