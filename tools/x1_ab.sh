#!/bin/bash
# x1 record-batch tests on the product library, then a same-box A/B of ab/ libraries on the blob workload
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_x1_fast_gpu.py tests/test_fastpath_gpu.py tests/test_compressor.py tests/test_rans_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/x1tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/x1tests.log
timeout -k 10 600 bash tools/ab_multi.sh "$AB_LIBS" --workload blob --no-secondary > gpurun_out/ab.log 2>&1
echo "ab rc=$?"
