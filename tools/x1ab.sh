#!/bin/bash
# x1 record-batch A/B: the x1 GPU tests on every library, then the blob bench per library
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LIBS=$1
: > gpurun_out/x1tests.log
for L in $LIBS; do
  echo "== $L" >> gpurun_out/x1tests.log
  ZR_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_x1_fast_gpu.py tests/test_rans_gpu.py tests/test_compressor.py -x -q --timeout 170 --timeout-method thread >> gpurun_out/x1tests.log 2>&1 || exit 1
done
timeout -k 10 600 bash tools/ab_multi.sh "$LIBS" --workload blob > gpurun_out/x1ab.log 2>&1
