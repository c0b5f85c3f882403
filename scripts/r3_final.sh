#!/bin/bash
# Round-3 evidence run (GPU box): GPU tests, the default bench (C2 + north-star / C3 lines), rocprofv3
# kernel stats per config, PMC traffic passes (FETCH_SIZE / WRITE_SIZE) for C2 and the north-star shape,
# one SQ pass per config.  Usage (repo root, on the box): bash scripts/r3_final.sh TAG
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-r3f}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest exit=$rc" >> $O/gpu_tests_$T.log; tail -3 $O/gpu_tests_$T.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 3;; esac
timeout -k 10 300 python bench.py > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed $?"; exit 4; }
echo "bench ok"
ARGS="--steps 300 --warmup 10 --no-cpu-baseline --extras 0 --other-steps 0 --targets 0 --latency-steps 300 --device-steps 300"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
for c in c2 ns c3 c5; do
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS > $O/bench_${c}_$T.json 2> $O/bench_${c}_$T.err || { echo "rocprof $c failed $?"; exit 5; }
    timeout -k 10 180 rocprofv3 --pmc $SQ --kernel-trace -d $O/sq_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS --device-steps 0 > $O/sq_${c}_$T.json 2> $O/sq_${c}_$T.err || { echo "sq $c failed $?"; exit 6; }
    echo "stats+sq $c ok"
done
for c in c2 ns; do
    timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmcf_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS --device-steps 0 --latency-steps 20 > $O/pmcf_${c}_$T.json 2> $O/pmcf_${c}_$T.err || { echo "pmcf $c failed $?"; exit 7; }
    timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmcw_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS --device-steps 0 --latency-steps 20 > $O/pmcw_${c}_$T.json 2> $O/pmcw_${c}_$T.err || { echo "pmcw $c failed $?"; exit 8; }
    echo "pmc $c ok"
done
echo ALLDONE
