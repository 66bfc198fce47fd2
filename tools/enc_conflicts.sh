#!/bin/bash
# LDS bank-conflict cycles and LDS instructions of k_enc_xn for the ab/
# libraries ($AB_LIBS), one counter pass each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/encc
for L in $AB_LIBS; do
  n=$(basename $L .so)
  ZR_LIB_PATH=$L timeout -s KILL 90 rocprofv3 --kernel-include-regex "k_enc_xn" --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/encc/$n -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/encc/$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
done
python3 tools/pmc_sum.py $(find gpurun_out/encc -name "*counter_collection.csv") > gpurun_out/encc/summary.txt 2>&1
cat gpurun_out/encc/summary.txt
