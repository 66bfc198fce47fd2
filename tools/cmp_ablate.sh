#!/bin/bash
# compaction ablations (diag build), headline workload, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for r in 1 2; do
  for A in 0 1 2 4 3 7; do
    ZR_CMP_ABL=$A ZR_LIB_PATH=zipora_amd/libzipora_amd_diag.so timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-host-path --no-secondary > gpurun_out/ab/run.log 2>&1 || { cat gpurun_out/ab/run.log; exit 1; }
    echo "CMP_ABL=$A: $(tail -1 gpurun_out/ab/run.log)"
  done
done
for r in 1 2; do
  for A in 0 1 2 3; do
    ZR_ABLATE=$A ZR_LIB_PATH=zipora_amd/libzipora_amd_diag.so timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-host-path --no-secondary > gpurun_out/ab/run.log 2>&1 || { cat gpurun_out/ab/run.log; exit 1; }
    echo "ENC_ABL=$A: $(tail -1 gpurun_out/ab/run.log)"
  done
done
