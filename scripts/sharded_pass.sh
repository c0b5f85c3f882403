#!/bin/bash
# World-1 sharded host steps timed from C (srbd_step_sharded over the xGMI exchange, bench.py --sharded): the per-rank
# shape of C5 on 8 GPUs (65 536 HyQReal rows) and the north-star shape.  Usage (repo root, GPU box): bash scripts/sharded_pass.sh TAG
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-sh}; mkdir -p $O
for w in "c5 65536" "ns 65536"; do
    set -- $w
    timeout -k 10 300 python bench.py --sharded --config $1 --num-samples $2 --steps 2000 --device-steps 1000 \
        > $O/sharded_${1}_${2}_$T.json 2> $O/sharded_${1}_${2}_$T.err || { echo "sharded $1 failed"; tail -5 $O/sharded_${1}_${2}_$T.err; exit 1; }
    python - $O/sharded_${1}_${2}_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["workload"], "value", d["value"], "ms", d["ms_per_step"], "p50", d["p50_step_ms"], "chain", d["device_chain"], d["kernels_us"])
PY
done
echo SHDONE
