#!/bin/bash
# PMC passes for the rANS kernels (run on the GPU box from the repo root).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path"
K="--kernel-include-regex k_dec_xn_fast|k_enc_xn|k_enc_compact|k_hist"
timeout -k 10 300 rocprofv3 $K --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc -o p1 -- $B > gpurun_out/pmc/p1.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d gpurun_out/pmc -o p2 -- $B > gpurun_out/pmc/p2.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o p3 -- $B > gpurun_out/pmc/p3.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o p4 -- $B > gpurun_out/pmc/p4.log 2>&1
timeout -k 10 300 rocprofv3 $K --kernel-trace --stats --output-format csv -d gpurun_out/pmc -o kt -- $B > gpurun_out/pmc/kt.log 2>&1
find gpurun_out/pmc -name "*.csv" | head -30
