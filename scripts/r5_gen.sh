#!/bin/bash
# Round-5 in-launch draws (GEN) at C5 (GPU box): parity tests, host A/B (SRBD_GEN=0 / default), the c5 bench
# line, then a rocprofv3 kernel trace of a short C5 run.  Each step under its own limit; stops at the first failure.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-g}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_regen.py "tests/test_gpu_fullsize.py" -x -q -o addopts="" \
    --timeout 240 --timeout-method thread -rf > $O/gen_tests_$T.log 2>&1
rc=$?; tail -3 $O/gen_tests_$T.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 400 python scripts/host_ab.py c5 500 rng=SRBD_GEN=0 rg0=SRBD_GEN_RG=0 rg8=SRBD_GEN_RG=8 rg16=SRBD_GEN_RG=16 rg24=SRBD_GEN_RG=24 rg36=SRBD_GEN_RG=36 > $O/gen_ab_$T.jsonl 2>&1 || { echo "ab failed"; tail -5 $O/gen_ab_$T.jsonl; exit 4; }
cat $O/gen_ab_$T.jsonl
timeout -k 10 300 python bench.py --config c5 --steps 500 --no-cpu-baseline --other-steps 0 > $O/gen_bench_$T.json 2> $O/gen_bench_$T.err || { echo bench failed; tail -5 $O/gen_bench_$T.err; exit 5; }
python - $O/gen_bench_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "p50", d.get("p50_step_ms"), "roofline", d["roofline"]["frac"], d["roofline"].get("kernel_us"), d.get("kernels_us"))
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gen_prof_$T -o run -- python3 $R/bench.py --config c5 --steps 200 --no-cpu-baseline --other-steps 0 --latency-steps 100 --device-steps 100 > $O/gen_prof_$T.log 2>&1 || { echo prof failed; tail -5 $O/gen_prof_$T.log; exit 6; }
find $O/gen_prof_$T -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -8'
echo ALLDONE
