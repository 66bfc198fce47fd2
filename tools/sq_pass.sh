#!/bin/bash
# SQ counters (two passes) of the headline kernels in the default bench shape:
#   bash tools/sq_pass.sh <out_dir> [bench args...]
set -o pipefail
O=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $O
K="--kernel-include-regex k_dec_xn_fast|k_enc_xn|k_enc_compact|k_hist|k_enc_x1_ring|k_dec_x1_fast|k_hist_small"
BP="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary $*"
timeout -s KILL 90 rocprofv3 $K --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/sq1 -o sq1 -- $BP > $O/sq1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 $K --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o sq2 -- $BP > $O/sq2.log 2>&1 || exit 1
python3 tools/pmc_sum.py $(find $O/sq1 $O/sq2 -name "*counter_collection.csv") > $O/sq_counters.txt 2>&1
echo "sq done"
