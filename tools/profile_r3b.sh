#!/bin/bash
# Round-3 profile, part B: HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes) and SQ counters.
set -e
R=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_$R
mkdir -p $O/summary
K="--kernel-include-regex k_dec_xn_fast|k_enc_xn|k_enc_compact|k_hist|k_fse_dec|k_fse_enc|k_copy16|k_enc_x1_fast|k_enc_x1_ring|k_dec_x1_fast|k_dec_x1_ring|k_hist_small"
BP="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary"
L="python3 bench.py --buffers 1 --buffer-mib 256 --no-cpu-baseline --no-host-path --no-secondary --steps 1 --warmup 1"
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 90 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_$n -o $n -- $BP > $O/pmc_$n.log 2>&1
  timeout -s KILL 90 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_lit_$n -o $n -- $L > $O/pmc_lit_$n.log 2>&1
  timeout -s KILL 120 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_fse_$n -o $n -- python3 bench.py --workload fse --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $O/pmc_fse_$n.log 2>&1
  timeout -s KILL 120 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_blob_$n -o $n -- python3 bench.py --workload blob --steps 1 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary > $O/pmc_blob_$n.log 2>&1
  timeout -s KILL 90 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_o1_$n -o $n -- python3 bench.py --workload o1 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $O/pmc_o1_$n.log 2>&1
done
timeout -s KILL 90 rocprofv3 $K --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/sq1 -o sq1 -- $BP > $O/sq1.log 2>&1
timeout -s KILL 90 rocprofv3 $K --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o sq2 -- $BP > $O/sq2.log 2>&1
python3 tools/pmc_sum.py $(find $O/sq1 $O/sq2 -name "*counter_collection.csv") > $O/summary/sq_counters.txt 2>&1 || true
echo done
