#!/bin/bash
# SQ counters for the fast rANS decoder and its ablations (ZR_DEC_ABL=0, 4, ...), two passes each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/dpmc; mkdir -p $O
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path"
K="--kernel-include-regex k_dec_xn_fast"
for v in "$@"; do
  ZR_ABLATE=0 ZR_DEC_ABL=$v timeout -k 10 120 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O -o v${v}_a -- $B > $O/v${v}_a.log 2>&1 || exit 1
  ZR_ABLATE=0 ZR_DEC_ABL=$v timeout -k 10 120 rocprofv3 $K --pmc SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d $O -o v${v}_b -- $B > $O/v${v}_b.log 2>&1 || exit 1
done
