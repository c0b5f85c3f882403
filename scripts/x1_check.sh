#!/bin/bash
# xGMI merge A/B (measurement; GPU box): SRBD_MERGE_STAGE=1 staged pass 1, 2 direct pass 1.
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for k in 1 2 1 2; do
  for m in xgmi local2; do
    SRBD_MERGE_STAGE=$k timeout -k 10 150 python scripts/sharded_probe.py $m > gpurun_out/x1_probe_${k}_$m.jsonl 2>gpurun_out/x1_probe_${k}_$m.err || { tail gpurun_out/x1_probe_${k}_$m.err; exit 4; }
    echo "stage=$k $(cat gpurun_out/x1_probe_${k}_$m.jsonl)"
  done
done
