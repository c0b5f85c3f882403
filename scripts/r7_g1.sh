R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > $O/gpu_tests_r7a.log 2>&1
rc=$?; tail -3 $O/gpu_tests_r7a.log; [ $rc -eq 0 ] || exit 3
for w in "c2 10000" "ns 65536"; do set -- $w
 timeout -k 10 120 python scripts/rollout_timeline.py $1 $2 > $O/tl_$1_r7a.json 2> $O/tl_$1_r7a.err || { echo "tl $1 failed"; exit 4; }
 timeout -k 10 120 python scripts/step_tail.py $1 $2 > $O/tail_$1_r7a.json 2> $O/tail_$1_r7a.err || { echo "tail $1 failed"; exit 5; }
done
cat $O/tl_*_r7a.json $O/tail_*_r7a.json
echo ALLDONE
