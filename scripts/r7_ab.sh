#!/bin/bash
# Library-variant A/B on the GPU box: host-to-host srbd_step p50 (scripts/host_ab.py) of the in-tree library ("cur")
# and each named variant (quadruped-pympc-tamols_amd/variants/lib_NAME.so), interleaved per workload.
# Usage: bash scripts/r7_ab.sh OUT.jsonl "WORKLOAD[:N] STEPS" ... -- NAME ...
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
out=$O/$1; shift
ws=(); while [ "$1" != "--" ]; do ws+=("$1"); shift; done; shift
for w in "${ws[@]}"; do set -- $w "${@}"
  wl=$1; st=$2; shift 2
  for rnd in 1 2; do
    for lib in cur "$@"; do L=$R/quadruped-pympc-tamols_amd/quadruped_pympc_amd/libsrbd_hip.so
      [ $lib != cur ] && L=$R/quadruped-pympc-tamols_amd/variants/lib_$lib.so
      SRBD_LIB_PATH=$L timeout -k 10 200 python scripts/host_ab.py $wl $st $lib=SRBD_NOP=$rnd >> $out || { echo "ab $wl $lib failed"; exit 3; }
    done
  done
done
cat $out
