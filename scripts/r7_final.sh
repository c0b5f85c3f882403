#!/bin/bash
# Final evidence (rounds 6-7) (GPU box): the full -m gpu suite, rocprofv3 kernel stats + PMC (FETCH / WRITE) + SQ for C2,
# north-star, C3 and C5 (scripts/evidence_pass.sh), the TAMOLS kernel at C4 (scripts/tamols_probe.py under
# rocprofv3), the chained C4 step (time split + kernel stats), SQ counters of the JAX-stream draws at the north-star
# shape, the per-rank C5 shape through the sharded step at world 1, the default bench line.  Each step under its
# own limit; stops at the first failure.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; T=${1:-r7z}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/gpu_tests_$T.log 2>&1
rc=$?; tail -3 $O/gpu_tests_$T.log; [ $rc -eq 0 ] || exit 3
bash scripts/evidence_pass.sh $T c2 ns c3 c5 || exit 4
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_c4_$T -o run --output-format csv -- python3 $R/scripts/tamols_probe.py > $O/tamols_probe_$T.json 2> $O/tamols_probe_$T.err || { echo tamols prof failed; exit 5; }
timeout -k 10 300 python scripts/c4_split_probe.py > $O/c4_split_$T.json 2> $O/c4_split_$T.err || { echo c4 split failed; exit 5; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_c4chain_$T -o run --output-format csv -- python3 $R/scripts/c4_split_probe.py 300 > /dev/null 2> $O/prof_c4chain_$T.err || { echo c4 chain prof failed; exit 5; }
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
RNGS=jax timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace -d $O/sq_jaxns_$T -o run --output-format csv -- python3 $R/scripts/jax_rng_time.py ns > $O/jaxns_$T.json 2> $O/jaxns_$T.err || { echo jax sq failed; exit 5; }
timeout -k 10 300 python bench.py --sharded --config c5 --num-samples 65536 --steps 1000 --no-cpu-baseline > $O/sharded_w1_c5rank_$T.json 2> $O/sharded_w1_c5rank_$T.err || { echo sharded failed; tail -5 $O/sharded_w1_c5rank_$T.err; exit 6; }
timeout -k 10 600 python bench.py > $O/bench_$T.json 2> $O/bench_$T.err || { echo bench failed; tail -5 $O/bench_$T.err; exit 7; }
echo ALLDONE
