#!/bin/bash
# rANS GPU parity tests, then the headline bench three times.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_rans_gpu.py tests/test_compressor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rc_tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/rc_bench_$r.log 2>&1 || exit 1
done
