#!/bin/bash
# Round 5: fused encode + compaction (k_enc_lb): parity tests, then same-box A/B
# of the default bench command (three alternations)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_enc_fused_gpu.py \
  tests/test_rans_r02_gpu.py::test_decode_errors_two_level_arrival tests/test_ref_asserts.py \
  > gpurun_out/r5_fused_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/r5_fused_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for F in 0 1; do
    timeout -k 10 120 python bench.py --enc-fused $F --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-secondary \
      > gpurun_out/r5_fused_ab_${F}_$i.json 2> gpurun_out/r5_fused_ab_${F}_$i.err || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/r5_fused_ab_${F}_$i.json').read().strip().splitlines()[-1])
print('fused=$F', d['value'], d['ms_per_step'], d['kernels_ms'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])"
  done
done
