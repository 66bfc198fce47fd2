#!/bin/bash
# Round 6: record decoder k_dec_x1_fast output group size (ZR_X1_XG) and line
# pairing (ZR_X1_PAIR): parity of each variant, same-box A/B of the record
# batch (configs[4]), FETCH/WRITE per dispatch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=zipora_amd/ab
O=gpurun_out/x1
mkdir -p $O
for L in $VARIANTS; do
  ZR_LIB_PATH=$A/lib_$L.so timeout -k 10 400 python -u -m pytest tests/test_x1_fast_gpu.py tests/test_fastpath_gpu.py tests/test_status_ws_gpu.py -x -q --timeout 170 --timeout-method thread > $O/tests_$L.log 2>&1 || { echo "tests failed: $L"; tail -5 $O/tests_$L.log; exit 1; }
done
for r in 1 2 3; do
  for L in base $VARIANTS; do
    ZR_LIB_PATH=$A/lib_$L.so timeout -k 10 200 python3 bench.py --workload blob --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary > $O/run.log 2>&1 || { cat $O/run.log; exit 1; }
    echo "$L: $(tail -1 $O/run.log)"
  done
done > $O/ab.log
for L in base $VARIANTS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    ZR_LIB_PATH=$A/lib_$L.so timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_dec_x1_fast|k_enc_x1_ring" --pmc $c --output-format csv -d $O/pmc_${L}_$c -o p -- python3 bench.py --workload blob --steps 1 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary > $O/pmc_${L}_$c.log 2>&1 || exit 1
  done
done
echo ok
