#!/bin/bash
# Round 3 (GPU box): GPU tests; C3 prefetch-window / grouping variants; C5 next-step draw placement.
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
O=gpurun_out; T=${1:-r3d}; mkdir -p $O; rm -f $O/variants.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest exit=$rc" >> $O/gpu_tests_$T.log; tail -3 $O/gpu_tests_$T.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 3;; esac
bash scripts/vrun.sh c3 cur cl2 cl3 cur=SRBD_GROUP_SIZE=32 || exit 2
for m in 0 3 1; do
  SRBD_NEXT_DRAWS=$m timeout -k 10 240 python bench.py --config c5 --steps 500 --warmup 20 --no-cpu-baseline --extras 0 --other-steps 0 --latency-steps 500 --device-steps 300 > $O/bench_c5_d${m}_$T.json 2> $O/bench_c5_d${m}_$T.err || { echo "bench c5 draws $m failed"; exit 4; }
  python -c "import json; d=json.loads(open('$O/bench_c5_d${m}_$T.json').read().strip().splitlines()[-1]); print('c5 draws $m', d['ms_per_step'], d['p50_step_ms'], d['kernels_us'])"
done
SRBD_FUSE_MAX=1048576 timeout -k 10 240 python bench.py --config c5 --steps 500 --warmup 20 --no-cpu-baseline --extras 0 --other-steps 0 --latency-steps 500 --device-steps 300 > $O/bench_c5_fuse_$T.json 2> $O/bench_c5_fuse_$T.err || exit 5
python -c "import json; d=json.loads(open('$O/bench_c5_fuse_$T.json').read().strip().splitlines()[-1]); print('c5 fused', d['ms_per_step'], d['p50_step_ms'], d['kernels_us'], d['device_chain'])"
echo PROBEDONE
