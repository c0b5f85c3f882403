#!/bin/bash
# Evidence pass on the GPU box: rocprofv3 kernel stats of short bench runs per config (c2, north-star, c3, c5),
# then per config the launch srbd_step issues (scripts/launch_probe.py, one kind of launch at a time) under a
# FETCH_SIZE pass, a WRITE_SIZE pass and one SQ pass, and at C2 the plain fused launch beside it (the KS A/B).
# Every step runs under its own time limit; the script stops at the first failure or GPU fault.
# Usage: bash scripts/evidence_pass.sh TAG [configs...]
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-ev}; shift; mkdir -p $O
CFGS=${@:-c2 ns c3 c5}
export TMPDIR=/tmp
fault() { grep -q -i -E 'illegal memory access|memory access fault|GPU fault|core dumped|error code 38' "$@"; }
step() {  # step NAME TIMEOUT cmd...  (stdout -> NAME.out, stderr -> NAME.err)
    local n=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$n.out 2> $O/$n.err
    local rc=$?
    if fault $O/$n.out $O/$n.err; then echo "GPU fault in $n"; exit 3; fi
    case $rc in 0) echo "$n ok";; *) echo "$n failed rc=$rc"; tail -5 $O/$n.err; exit 4;; esac
}
ARGS="--steps 300 --warmup 10 --no-cpu-baseline --extras 0 --other-steps 0 --targets 0 --latency-steps 300 --device-steps 300"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
for c in $CFGS; do
    step stats_${c}_$T 180 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$T -o run --output-format csv -- python3 $R/bench.py --config $c $ARGS
    L="launch_probe.py $c step 300"
    step pmcf_${c}_$T 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmcf_${c}_$T -o run --output-format csv -- python3 $R/scripts/$L
    step pmcw_${c}_$T 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmcw_${c}_$T -o run --output-format csv -- python3 $R/scripts/$L
    step sq_${c}_$T 120 rocprofv3 --pmc $SQ --kernel-trace -d $O/sq_${c}_$T -o run --output-format csv -- python3 $R/scripts/$L
done
case " $CFGS " in *" c2 "*)  # the KS A/B at C2: the plain rollout + next-step draws, alone
    L="launch_probe.py c2 fused 300"
    step pmcf_c2fused_$T 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmcf_c2fused_$T -o run --output-format csv -- python3 $R/scripts/$L
    step pmcw_c2fused_$T 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmcw_c2fused_$T -o run --output-format csv -- python3 $R/scripts/$L
    step stats_c2fused_$T 120 rocprofv3 --kernel-trace --stats -d $O/prof_c2fused_$T -o run --output-format csv -- python3 $R/scripts/$L
    ;;
esac
echo ALLDONE
