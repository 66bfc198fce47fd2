#!/bin/bash
# FSE parity tests (FSE, PA-Zip stage, compressor) then the configs[2] bench at 64 and 16 KiB blocks.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_fse_gpu.py tests/test_pazip.py tests/test_compressor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fse_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --workload fse --no-cpu-baseline > gpurun_out/fse_bench.log 2>&1 && \
timeout -k 10 200 python -u bench.py --workload fse --fse-block-kib 16 --no-cpu-baseline > gpurun_out/fse16_bench.log 2>&1
