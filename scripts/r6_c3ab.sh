#!/bin/bash
# C3 A/B on the GPU box: the step input by value (KS) against the upload kernel (SRBD_KS=0); bench line + rocprof.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O; T=${1:-ab}
ARGS="--config c3 --steps 2000 --targets 0 --extras 0 --no-cpu-baseline --other-steps 0 --device-steps 300"
for ks in 1 0; do
  SRBD_KS=$ks timeout -k 10 200 python bench.py $ARGS > $O/bench_${T}_ks$ks.json 2> $O/bench_${T}_ks$ks.err || { echo "bench failed"; tail -5 $O/bench_${T}_ks$ks.err; exit 4; }
  python - "$O/bench_${T}_ks$ks.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1][-12:], "p50", d["p50_step_ms"], "kernels", d["kernels_us"])
PY
done
cd /tmp && export TMPDIR=/tmp
for ks in 1 0; do
  SRBD_KS=$ks timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_${T}_ks$ks -o run --output-format csv -- python3 $R/bench.py $ARGS --steps 300 > /dev/null 2> $O/prof_${T}_ks$ks.err || { echo prof failed; exit 5; }
done
echo DONE
