#!/bin/bash
# Round-4: record decoder with 32-step tiles (product build) - x1 tests, then a
# same-box blob A/B of ab/lib_t16.so (16-step tiles) against ab/lib_t32.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/x1t32
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_x1_fast_gpu.py tests/test_fastpath_gpu.py tests/test_compressor.py tests/test_rans_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > $O/tests.log 2>&1 && echo "tests ok" || { tail -30 $O/tests.log; exit 1; }
ROUNDS=3 timeout -k 10 600 bash tools/ab_multi.sh "zipora_amd/ab/lib_t16.so zipora_amd/ab/lib_t32.so" --workload blob > $O/ab_blob.log 2>&1 && echo "ab ok" && python3 tools/ab_summary.py $O/ab_blob.log
