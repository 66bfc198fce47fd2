#!/bin/bash
# Round 5: decoder prologue merge + encoder plain loads: parity, then same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rans_r02_gpu.py \
  tests/test_fastpath_gpu.py tests/test_rans_gpu.py tests/test_graph_capture_gpu.py > gpurun_out/r5_ab2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_ab2_tests.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=4 bash tools/ab_multi.sh "zipora_amd/ab/lib_base.so zipora_amd/ab/lib_encT.so zipora_amd/ab/lib_mrg.so" --no-secondary > gpurun_out/r5_ab2.log 2>&1
rc=$?; echo "ab rc=$rc"
python3 tools/ab_summary.py gpurun_out/r5_ab2.log 2>/dev/null || cut -c1-300 gpurun_out/r5_ab2.log
