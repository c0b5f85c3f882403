#!/bin/bash
# Last check of the final tree (GPU box): smoke(), the -m gpu suite, the default bench line.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-r7w}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 || { echo smoke failed; tail -5 $O/smoke_$T.log; exit 2; }
tail -1 $O/smoke_$T.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/gpu_tests_$T.log 2>&1
rc=$?; tail -2 $O/gpu_tests_$T.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 600 python bench.py > $O/bench_$T.json 2> $O/bench_$T.err || { echo bench failed; tail -5 $O/bench_$T.err; exit 4; }
python -c "
import json; d=json.load(open('$O/bench_$T.json'))
print({k: d[k] for k in ('value', 'p50_step_ms')}, {k: (d[k].get('p50_ms') or d[k].get('p50_step_ms')) for k in ('interface_step', 'c4', 'north_star_65536', 'c3', 'c5_1gpu')})"
echo ALLDONE
