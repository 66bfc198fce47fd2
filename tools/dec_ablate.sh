#!/bin/bash
# Decoder ablations on the diagnostic build (ZR_DEC_ABL: 1 no output stores,
# 2 no slot-table read, 4 no refills, 7 all three), headline workload, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for r in 1 2; do
  for A in ${DEC_ABLS:-0 1 2 4 7}; do
    ZR_DEC_ABL=$A ZR_LIB_PATH=zipora_amd/libzipora_amd_diag.so timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-host-path "$@" > gpurun_out/ab/run.log 2>&1 || { cat gpurun_out/ab/run.log; exit 1; }
    echo "DEC_ABL=$A $*: $(tail -1 gpurun_out/ab/run.log)"
  done
done
