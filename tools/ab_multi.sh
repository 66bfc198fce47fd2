#!/bin/bash
# Same-box A/B of several library builds (kernel times from the diagnostic JSON line):
#   bash tools/ab_multi.sh "<lib.so> <lib.so> ..." [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
LIBS=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-3}); do
  for L in $LIBS; do
    ZR_LIB_PATH=$L timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path "$@" \
      > gpurun_out/ab/run.log 2>&1 || { cat gpurun_out/ab/run.log; exit 1; }
    echo "$(basename $L) $*: $(tail -1 gpurun_out/ab/run.log)"
  done
done
