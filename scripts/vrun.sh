#!/bin/bash
# Variant probes on the GPU box: scripts/vrun.sh CONFIGS NAME[=ENV=VAL,...] ...
#   NAME "cur" = the in-tree library; other names = quadruped-pympc-tamols_amd/variants/lib_NAME.so
cd ${GRAFT_REPO_ROOT:-/root/repo}
cfgs=$1; shift
for spec in "$@"; do
  name=${spec%%=*}; envs=""; [ "$spec" != "$name" ] && envs=${spec#*=}
  lib=$PWD/quadruped-pympc-tamols_amd/variants/lib_$name.so
  [ "$name" = "cur" ] && lib=$PWD/quadruped-pympc-tamols_amd/quadruped_pympc_amd/libsrbd_hip.so
  env SRBD_LIB_PATH=$lib ${envs//,/ } timeout -k 10 180 python scripts/variant_probe.py "$spec" $cfgs >> gpurun_out/variants.jsonl || exit 1
done
echo VDONE
