#!/bin/bash
# rANS/compressor GPU parity tests, then the configs[4] record-batch bench twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_rans_gpu.py tests/test_compressor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bc_tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --workload blob --no-cpu-baseline --no-host-path > gpurun_out/bc_bench_$r.log 2>&1 || exit 1
done
