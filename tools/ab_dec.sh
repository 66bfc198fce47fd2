#!/bin/bash
# A/B of a k_dec_xn_fast variant (ZR_DEC_ABL=$1): rANS GPU parity tests under
# the variant, then the headline bench with the product kernel and the variant.
set -o pipefail
V=${1:-16}
cd $GRAFT_REPO_ROOT
ZR_DEC_ABL=$V timeout -k 10 300 python -u -m pytest tests/test_rans_gpu.py tests/test_compressor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/ab_base.log 2>&1 && \
ZR_DEC_ABL=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/ab_var.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/ab_base2.log 2>&1 && \
ZR_DEC_ABL=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/ab_var2.log 2>&1
