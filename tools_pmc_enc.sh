#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmce
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path"
K="--kernel-include-regex k_enc_xn|k_dec_fast|k_enc_compact"
timeout -k 10 300 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR --output-format csv -d gpurun_out/pmce -o e1 -- $B > gpurun_out/pmce/e1.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmce -o e2 -- $B > gpurun_out/pmce/e2.log 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > gpurun_out/pmce/bench_normal.log 2>&1
ZR_ABLATE=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > gpurun_out/pmce/bench_nostore.log 2>&1 || true
tail -1 gpurun_out/pmce/bench_normal.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('normal', d['kernels_ms'])"
tail -1 gpurun_out/pmce/bench_nostore.log | tail -c 600
