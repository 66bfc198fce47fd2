#!/bin/bash
# Round 6: the 1024-lane decoder with 4-byte slot entries and the ring's mirror
# row (ZR_DEC_T8=0) against the 8-byte default: same-box A/B, parity, SQ counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=zipora_amd/ab
mkdir -p gpurun_out/t4
ROUNDS=5 bash tools/ab_multi.sh "$A/lib_base.so $A/lib_t4.so" --no-secondary > gpurun_out/t4/ab.log 2>&1 && \
ZR_LIB_PATH=$A/lib_t4.so timeout -k 10 300 python -u -m pytest tests/test_rans_r02_gpu.py tests/test_fastpath_gpu.py tests/test_status_ws_gpu.py -x -q --timeout 170 --timeout-method thread > gpurun_out/t4/tests.log 2>&1 && \
for L in base t4; do
  ZR_LIB_PATH=$A/lib_$L.so timeout -s KILL 90 rocprofv3 --kernel-include-regex "k_dec_xn_fast|k_enc_xn" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/t4/sq_$L -o sq -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary > gpurun_out/t4/sq_$L.log 2>&1 || exit 1
  ZR_LIB_PATH=$A/lib_$L.so timeout -s KILL 90 rocprofv3 --kernel-include-regex "k_dec_xn_fast|k_enc_xn" --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/t4/sq2_$L -o sq -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary > gpurun_out/t4/sq2_$L.log 2>&1 || exit 1
done
echo ok
