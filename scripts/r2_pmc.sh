#!/bin/bash
# PMC passes over a short C2 bench (one counter group per pass, normal SIGTERM timeouts), plus one
# with the supplementary TAMOLS / interface probes (the round-1 stall candidate).
# Usage (repo root, on the box): bash scripts/r2_pmc.sh TAG
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-pmc}; mkdir -p $O
export TMPDIR=/tmp
ARGS="--steps 200 --warmup 5 --no-cpu-baseline --latency-steps 20 --device-steps 0 --other-steps 0"
pass() {  # name, counters, extra bench args
    local n=$1 c=$2; shift 2
    local t0=$(date +%s.%N)
    timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace -d $O/${n}_$T -o run --output-format csv -- python3 $R/bench.py $ARGS "$@" > $O/${n}_$T.json 2> $O/${n}_$T.err
    local rc=$?
    echo "$n rc=$rc wall=$(echo "$(date +%s.%N) - $t0" | bc) marker=$(grep -c 'body done' $O/${n}_$T.err)"
    return $rc
}
pass sqa "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" --extras 0 || exit 2
pass sqb "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" --extras 0 || exit 3
pass pmcf "FETCH_SIZE" --extras 0 || exit 4
pass pmcw "WRITE_SIZE" --extras 0 || exit 5
pass pmcx "FETCH_SIZE" --extras 20 || exit 6
echo ALLDONE
