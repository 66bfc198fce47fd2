#!/bin/bash
# Parity tests and the headline bench once per argument, each run with ZR_CMP_VAR set to it
# (a hook for A/B builds that read it; the committed kernels ignore it).
set -o pipefail
cd $GRAFT_REPO_ROOT
for V in "$@"; do
  ZR_CMP_VAR=$V timeout -k 10 200 python -u -m pytest tests/test_rans_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cmp_tests_$V.log 2>&1 || exit 1
  ZR_CMP_VAR=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/cmp_bench_$V.log 2>&1 || exit 1
done
