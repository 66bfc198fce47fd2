#!/bin/bash
# Round-4: the encoder's exact next-piece wait (ZR_ENC_VW): encoder parity tests
# on the product build, then a same-box A/B of ab/lib_novw.so against ab/lib_vw.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/vw
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_rans_r02_gpu.py tests/test_enc_v2_gpu.py tests/test_enc_split_gpu.py tests/test_fastpath_gpu.py tests/test_rans_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > $O/tests.log 2>&1 && echo "tests ok" || { tail -30 $O/tests.log; exit 1; }
ROUNDS=3 timeout -k 10 600 bash tools/ab_multi.sh "zipora_amd/ab/lib_novw.so zipora_amd/ab/lib_vw.so" > $O/ab.log 2>&1 && echo "ab ok" && python3 tools/ab_summary.py $O/ab.log
ROUNDS=2 timeout -k 10 600 bash tools/ab_multi.sh "zipora_amd/ab/lib_novw.so zipora_amd/ab/lib_vw.so" --workload blob > $O/ab_blob.log 2>&1 && echo "ab blob ok" && python3 tools/ab_summary.py $O/ab_blob.log
