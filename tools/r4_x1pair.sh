#!/bin/bash
# Round-4: the record encoder's paired input-line loads (ab/lib_x1pair.so) against
# the product (ab/lib_base.so): x1 parity tests on the variant, same-box blob A/B,
# FETCH_SIZE / WRITE_SIZE of the record kernels for both
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/x1pair
mkdir -p $O
ZR_LIB_PATH=zipora_amd/ab/lib_x1pair.so timeout -k 10 300 python -u -m pytest tests/test_x1_fast_gpu.py tests/test_fastpath_gpu.py tests/test_enc_v2_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > $O/tests.log 2>&1 && echo "tests ok" && \
ROUNDS=3 timeout -k 10 600 bash tools/ab_multi.sh "zipora_amd/ab/lib_base.so zipora_amd/ab/lib_x1pair.so" --workload blob > $O/ab_blob.log 2>&1 && echo "ab ok" && \
for L in base x1pair; do
  for c in FETCH_SIZE WRITE_SIZE; do
    ZR_LIB_PATH=zipora_amd/ab/lib_$L.so timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_enc_x1_ring|k_dec_x1_fast|k_hist_small" --pmc $c --output-format csv -d $O/pmc_${L}_$c -o p -- python3 bench.py --workload blob --steps 1 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary > $O/pmc_${L}_$c.log 2>&1 || { echo "pmc $L $c failed"; exit 1; }
  done
done && python3 tools/pmc_sum.py $(find $O -name "*counter_collection.csv") > $O/pmc_summary.txt 2>&1; echo done
