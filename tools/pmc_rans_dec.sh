#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcd
rocprofv3 -L > gpurun_out/pmcd/counters.txt 2>&1 || true
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path"
K="--kernel-include-regex k_dec_xn_fast|k_enc_xn"
timeout -k 10 300 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcd -o d1 -- $B > gpurun_out/pmcd/d1.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_WAVES --output-format csv -d gpurun_out/pmcd -o d2 -- $B > gpurun_out/pmcd/d2.log 2>&1
ls gpurun_out/pmcd
