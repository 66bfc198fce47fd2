#!/bin/bash
# x1 decoder A/B: tests on the first library, then blob bench per library
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LIBS=$1
FIRST=${LIBS%% *}
ZR_LIB_PATH=$FIRST timeout -k 10 300 python -u -m pytest tests/test_x1_fast_gpu.py tests/test_rans_gpu.py -x -q --timeout 170 --timeout-method thread > gpurun_out/x1tests.log 2>&1 && \
timeout -k 10 600 bash tools/ab_multi.sh "$LIBS" --workload blob > gpurun_out/x1ab.log 2>&1
