#!/bin/bash
# Round-3 (second half) evidence run on the GPU box: GPU tests, the default bench, rocprofv3 kernel stats and
# one SQ counter pass per config (C2, north-star, C3, C5), FETCH_SIZE / WRITE_SIZE passes for C2 and the
# north-star shape, the world-1 sharded probe at the per-rank 8-GPU C5 shape.  Every step runs under its own
# time limit and the script stops at the first failure or GPU fault.  Usage: bash scripts/r3m_final.sh TAG
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-r3m}; mkdir -p $O
export TMPDIR=/tmp
fault() { grep -q -i -E 'illegal memory access|memory access fault|GPU fault|core dumped|error code 38' "$@"; }
step() {  # step NAME TIMEOUT cmd...  (stdout -> NAME.out, stderr -> NAME.err)
    local n=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$n.out 2> $O/$n.err
    local rc=$?
    if fault $O/$n.out $O/$n.err; then echo "GPU fault in $n"; exit 3; fi
    case $rc in 0) echo "$n ok";; *) echo "$n failed rc=$rc"; tail -5 $O/$n.err; exit 4;; esac
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest exit=$rc" >> $O/gpu_tests_$T.log; tail -3 $O/gpu_tests_$T.log
if fault $O/gpu_tests_$T.log; then echo "GPU fault in tests"; exit 3; fi
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 3;; esac
step bench_$T 300 python bench.py
ARGS="--steps 300 --warmup 10 --no-cpu-baseline --extras 0 --other-steps 0 --targets 0 --latency-steps 300 --device-steps 300"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
for c in c2 ns c3 c5; do
    step bench_${c}_$T 180 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS
    step sq_${c}_$T 180 rocprofv3 --pmc $SQ --kernel-trace -d $O/sq_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS --device-steps 0
done
for c in c2 ns; do
    step pmcf_${c}_$T 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmcf_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS --device-steps 0 --latency-steps 20
    step pmcw_${c}_$T 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmcw_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS --device-steps 0 --latency-steps 20
done
SHARD_CFG=ns step shard_ns_$T 150 python scripts/sharded_probe.py xgmi
echo ALLDONE
