#!/bin/bash
# Round-7 experiment: quad permutations through ds_swizzle (SRBD_XS=1 variant) against DPP; swizzle/DPP unit costs.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o /tmp/sp scripts/swizzle_probe.hip 2>/dev/null && timeout -k 10 120 /tmp/sp > $O/swizzle_r7.jsonl || exit 2
cat $O/swizzle_r7.jsonl
CUR=$R/quadruped-pympc-tamols_amd/quadruped_pympc_amd/libsrbd_hip.so
XS=$R/quadruped-pympc-tamols_amd/variants/lib_xs.so
for w in "ns:65536 2000" "c2 3000" "c3 1000"; do set -- $w
  for lib in cur xs; do L=$CUR; [ $lib = xs ] && L=$XS
    SRBD_LIB_PATH=$L timeout -k 10 200 python scripts/host_ab.py $1 $2 $lib=SRBD_NOP=1 >> $O/ab_xs.jsonl || { echo "ab $1 $lib failed"; exit 3; }
  done
done
cat $O/ab_xs.jsonl
SRBD_LIB_PATH=$XS timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -o addopts="" --timeout 120 --timeout-method thread > $O/xs_parity.log 2>&1; tail -2 $O/xs_parity.log
