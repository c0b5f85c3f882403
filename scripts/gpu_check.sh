#!/bin/bash
# One GPU-box session: GPU tests, the default bench, and a rocprofv3 kernel trace of a short bench.
# Usage (from the repo root, on the box): bash scripts/gpu_check.sh TAG
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-run}; mkdir -p $O
timeout -k 10 500 python -m pytest tests -m gpu -q -o addopts="" --timeout 240 -rf > $O/gpu_tests_$T.log 2>&1
echo "pytest exit=$?" >> $O/gpu_tests_$T.log
rc=$(tail -1 $O/gpu_tests_$T.log)
case "$rc" in *"exit=0"|*"exit=1") ;; *) echo "stopping after $rc"; exit 3;; esac
timeout -k 10 300 python scripts/kernel_sweep.py c2 c3 10000 65536 262144 > $O/sweep_$T.jsonl 2> $O/sweep_$T.err || { echo "sweep failed $?"; exit 6; }
timeout -k 10 300 python bench.py --steps 2000 --warmup 20 > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed $?"; exit 4; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 300 --no-cpu-baseline --latency-steps 50 > $O/bench_prof_$T.json 2> $O/bench_prof_$T.err || { echo "rocprof failed $?"; exit 5; }
# HBM traffic: FETCH_SIZE and WRITE_SIZE need separate passes (TCC slots); --kernel-trace only
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmcf_$T -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 5 --no-cpu-baseline --latency-steps 20 > $O/pmcf_$T.json 2> $O/pmcf_$T.err || { echo "pmc fetch failed $?"; exit 7; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmcw_$T -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 5 --no-cpu-baseline --latency-steps 20 > $O/pmcw_$T.json 2> $O/pmcw_$T.err || { echo "pmc write failed $?"; exit 8; }
python3 scripts/pmc_summary.py $O/pmcf_$T $O/pmcw_$T go2_trot_flat_mppi_n10000_h12_zo $O/pmc_traffic_$T.json > $O/pmc_summary_$T.log 2>&1 || echo "pmc summary failed (see log)"
echo ALLDONE
