#!/bin/bash
# SQ issue/wait counters for the x1 record-batch coder kernels (blob workload)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sqx1
B="python3 bench.py --workload blob --steps 1 --warmup 1 --no-cpu-baseline --no-host-path"
K="--kernel-include-regex k_dec_x1_ring|k_enc_x1_fast"
timeout -k 10 300 rocprofv3 $K --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/sqx1 -o s1 -- $B > gpurun_out/sqx1/s1.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sqx1 -o s2 -- $B > gpurun_out/sqx1/s2.log 2>&1
