#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_x1_fast_gpu.py tests/test_rans_gpu.py tests/test_compressor.py -x -v --timeout 170 --timeout-method thread > gpurun_out/x1tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload blob --no-cpu-baseline --no-host-path > gpurun_out/bench_blob_x1.log 2>&1
