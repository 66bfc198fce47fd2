#!/bin/bash
# Decoder output-store policy A/B: rANS parity under ZR_DEC_ABL=16 (nt stores), the
# alternating bench, then FETCH_SIZE of k_dec_xn_fast for both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ZR_DEC_ABL=16 timeout -k 10 300 python -u -m pytest tests/test_rans_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nt_tests.log 2>&1 || exit 1
bash tools/ab_env.sh ZR_DEC_ABL=16 || exit 1
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path"
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_dec_xn_fast --pmc FETCH_SIZE --output-format csv -d gpurun_out/nt_base -o f -- $B > gpurun_out/nt_base.log 2>&1 || exit 1
export ZR_DEC_ABL=16
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_dec_xn_fast --pmc FETCH_SIZE --output-format csv -d gpurun_out/nt_var -o f -- $B > gpurun_out/nt_var.log 2>&1
