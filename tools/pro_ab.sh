#!/bin/bash
# Prologue/setup round-trip changes: rANS GPU tests on the working-tree
# library, then a same-box A/B of HEAD's library (lib_base) against the
# variant (lib_var), both built by tools/build_wt.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fastpath_gpu.py tests/test_rans_gpu.py tests/test_rans_r02_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/pro_tests.log 2>&1 && \
bash tools/ab_multi.sh "zipora_amd/ab/lib_base.so $(for v in ${@:-var}; do echo -n "zipora_amd/ab/lib_$v.so "; done)"
