#!/bin/bash
# fast-path tests on the product library, then same-box A/B of ab/ libraries
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fastpath_gpu.py tests/test_rans_r02_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/fastpath.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/fastpath.log
timeout -k 10 600 bash tools/ab_multi.sh "$AB_LIBS" > gpurun_out/ab.log 2>&1
echo "ab rc=$?"
