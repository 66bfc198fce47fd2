#!/bin/bash
# SQ counters and kernel-trace stats of the encoder at both widths
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/wpmc
mkdir -p $O
K="--kernel-include-regex k_enc_xn|k_enc_compact"
for w in 256 512 1024; do
  BP="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary --enc-width $w"
  timeout -s KILL 90 rocprofv3 $K --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/sq1_$w -o sq1 -- $BP > $O/sq1_$w.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 $K --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/sq2_$w -o sq2 -- $BP > $O/sq2_$w.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$w -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-secondary --enc-width $w > $O/kt_$w.log 2>&1 || exit 1
done
python3 tools/pmc_sum.py $(find $O -name "*counter_collection.csv" | sort) > $O/summary.txt 2>&1
for w in 256 512 1024; do echo "== $w"; grep -E "k_enc_xn|k_enc_compact|k_dec_xn|k_hist" $(find $O/kt_$w -name "*kernel_stats.csv") | cut -d, -f1-5; done >> $O/summary.txt
echo done
