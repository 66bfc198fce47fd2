#!/bin/bash
# rANS decode diagnostics: ablation timings (ZR_DEC_ABL) and SQ counter passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/diag; mkdir -p $O
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-path"
for a in 0 1 2 4 3 7; do
  ZR_ABLATE=0 ZR_DEC_ABL=$a timeout -k 10 120 $B > $O/abl_$a.log 2>&1 || exit 1
done
K="--kernel-include-regex k_dec_xn_fast"
timeout -k 10 120 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O -o p1 -- $B > $O/p1.log 2>&1 && \
timeout -k 10 120 rocprofv3 $K --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O -o p2 -- $B > $O/p2.log 2>&1 && \
timeout -k 10 120 rocprofv3 $K --pmc SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_IFETCH --output-format csv -d $O -o p3 -- $B > $O/p3.log 2>&1
