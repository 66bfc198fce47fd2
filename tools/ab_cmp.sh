#!/bin/bash
# A/B of k_enc_compact_lds shapes (ZR_CMP_VAR): parity tests and the headline bench per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
for V in "$@"; do
  ZR_CMP_VAR=$V timeout -k 10 200 python -u -m pytest tests/test_rans_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cmp_tests_$V.log 2>&1 || exit 1
  ZR_CMP_VAR=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/cmp_bench_$V.log 2>&1 || exit 1
done
