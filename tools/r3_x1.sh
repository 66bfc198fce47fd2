#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_x1_fast_gpu.py tests/test_fastpath_gpu.py tests/test_compressor.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/x1tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/x1tests.log
timeout -k 10 500 bash tools/ab_multi.sh "zipora_amd/ab/lib_x1old.so zipora_amd/ab/lib_x1new.so" --workload blob --no-secondary > gpurun_out/ab.log 2>&1
echo "ab rc=$?"
