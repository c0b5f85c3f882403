R=${GRAFT_REPO_ROOT:-/root/repo}; cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out; mkdir -p $O
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
timeout -k 10 120 python3 $R/scripts/jax_rng_time.py ns > $O/jaxt.json 2> $O/jaxt.err || { echo fail1; tail -5 $O/jaxt.err; exit 3; }
cat $O/jaxt.json
RNGS=jax timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace -d $O/sq_jax -o run --output-format csv -- python3 $R/scripts/jax_rng_time.py ns > $O/jaxsq.out 2> $O/jaxsq.err || { echo fail2; tail -5 $O/jaxsq.err; exit 4; }
python3 $R/scripts/sq_summary.py $O/sq_jax $O/sq_jax.json
