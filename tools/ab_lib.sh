#!/bin/bash
# Same-box A/B of two library builds on a bench workload (kernel times from the
# diagnostic JSON line). Usage on the GPU box:
#   bash tools/ab_lib.sh <libA.so> <libB.so> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
A=$1; B=$2; shift 2
mkdir -p gpurun_out/ab
for r in 1 2; do
  for L in "$A" "$B"; do
    ZR_LIB_PATH=$L timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path "$@" \
      > gpurun_out/ab/run.log 2>&1 || { cat gpurun_out/ab/run.log; exit 1; }
    echo "$(basename $L) $*: $(tail -1 gpurun_out/ab/run.log)"
  done
done
