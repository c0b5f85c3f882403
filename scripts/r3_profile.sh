#!/bin/bash
# Round-3 profiles of the throughput shapes: rocprofv3 kernel stats and one SQ counter pass per config.
# Usage (repo root, on the box): bash scripts/r3_profile.sh TAG [configs...]   (default: ns c3 c5)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-r3}; shift; mkdir -p $O
CFGS=${@:-ns c3 c5}
export TMPDIR=/tmp
ARGS="--steps 300 --warmup 10 --no-cpu-baseline --extras 0 --other-steps 0 --latency-steps 300 --device-steps 300"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
for c in $CFGS; do
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS > $O/bench_${c}_$T.json 2> $O/bench_${c}_$T.err || { echo "rocprof $c failed $?"; exit 2; }
    echo "stats $c ok"
    timeout -k 10 180 rocprofv3 --pmc $SQ --kernel-trace -d $O/sq_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS --device-steps 0 > $O/sq_${c}_$T.json 2> $O/sq_${c}_$T.err || { echo "sq $c failed $?"; exit 3; }
    echo "sq $c ok"
done
echo ALLDONE
