#!/bin/bash
# Round-2 GPU-box session: all GPU tests, the default bench, C5 on one GPU, a rocprofv3 kernel trace.
# Usage (repo root, on the box): bash scripts/r2_check.sh TAG [pytest args...]
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-r2}; shift; mkdir -p $O
TESTS=${@:-tests -m gpu}
echo "nproc=$(nproc) affinity=$(python3 -c 'import os;print(len(os.sched_getaffinity(0)))') omp=$OMP_NUM_THREADS cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)" > $O/host_$T.txt
timeout -k 10 600 python -u -m pytest $TESTS -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/gpu_tests_$T.log 2>&1
rc=$?
echo "pytest exit=$rc" >> $O/gpu_tests_$T.log
tail -3 $O/gpu_tests_$T.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 3;; esac
timeout -k 10 240 python bench.py --steps 2000 --warmup 20 > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed $?"; exit 4; }
cat $O/bench_$T.json
timeout -k 10 180 python bench.py --config c5 --steps 300 --warmup 10 --cpu-seconds 10 --extras 0 > $O/bench_c5_$T.json 2> $O/bench_c5_$T.err || { echo "bench c5 failed $?"; exit 5; }
cat $O/bench_c5_$T.json
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 1000 --warmup 20 --no-cpu-baseline --extras 0 > $O/bench_prof_$T.json 2> $O/bench_prof_$T.err || { echo "rocprof failed $?"; exit 6; }
echo ALLDONE
