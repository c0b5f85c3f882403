cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
T=${1:-r3c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -o addopts="" --timeout 240 --timeout-method thread -rf > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_$T.log
case "$rc" in 0|1) ;; *) echo "pytest rc=$rc"; exit 3;; esac
shift
[ $# -gt 0 ] && { bash scripts/vrun.sh "$@" || exit 4; }
echo R3CDONE
