#!/bin/bash
# compaction ablations on the current kernel (diag build), headline workload, same box:
# 0 product, 1 no phase-2 stores, 2 no LDS image writes, 4 loads of one 256-B run, 7 none of the three
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for A in 0 1 2 4 7; do
    ZR_CMP_ABL=$A ZR_LIB_PATH=zipora_amd/libzipora_amd_diag.so timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-host-path --no-secondary > gpurun_out/ab/run.log 2>&1 || { cat gpurun_out/ab/run.log; exit 1; }
    echo "CMP_ABL=$A: $(tail -1 gpurun_out/ab/run.log)"
  done
done
