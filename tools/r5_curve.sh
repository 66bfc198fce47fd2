#!/bin/bash
# Round 5: new parity tests, then the decoder frac-vs-N curve on ONE 256 MiB
# uniform buffer (N = 2^18, 2^19, 2^20) for both decoder rings.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_fastpath_gpu.py::test_dma_ring_decoder tests/test_fastpath_gpu.py::test_single_buffer_many_streams \
  tests/test_rans_r02_gpu.py::test_decode_errors_two_level_arrival tests/test_ref_asserts.py \
  > gpurun_out/r5_tests.log 2>&1
echo "tests rc=$?"
tail -5 gpurun_out/r5_tests.log
for N in 262144 524288 1048576; do
  for R in 1 2; do
    timeout -k 10 120 python bench.py --buffers 1 --buffer-mib 256 --streams $N --dec-ring $R --steps 10 --warmup 2 \
      --no-cpu-baseline --no-host-path --no-secondary > gpurun_out/r5_curve_${N}_${R}.json 2> gpurun_out/r5_curve_${N}_${R}.err
    echo "N=$N ring=$R rc=$?"
  done
done
