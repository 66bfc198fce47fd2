#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the headline decoder for the ab/ libraries ($AB_LIBS), one counter pass each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc3
for L in $AB_LIBS; do
  n=$(basename $L .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    ZR_LIB_PATH=$L timeout -s KILL 90 rocprofv3 --kernel-include-regex "k_dec_xn_fast|k_enc_xn|k_enc_compact|k_hist" --pmc $c --output-format csv -d gpurun_out/pmc3/${n}_$c -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/pmc3/${n}_$c.log 2>&1 || { echo "pmc $n $c failed"; exit 1; }
  done
done
python3 tools/pmc_sum.py $(find gpurun_out/pmc3 -name "*counter_collection.csv") > gpurun_out/pmc3/summary.txt 2>&1
echo pmc done
