#!/bin/bash
# One gpurun call for a same-box A/B of library builds (tools/build_wt.sh makes
# zipora_amd/ab/lib_<name>.so from the working tree, optionally patched):
#   gpurun -- 'bash tools/gpu_ab.sh "<lib.so> <lib.so> ..." [tests]'
# The GPU parity tests run first when the second argument is "tests".
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LIBS=$1
if [ "$2" = "tests" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
fi
timeout -k 10 400 bash tools/ab_multi.sh "$LIBS" > gpurun_out/ab1.log 2>&1 && \
timeout -k 10 400 bash tools/ab_multi.sh "$LIBS" --buffers 1 --buffer-mib 256 --steps 4 >> gpurun_out/ab1.log 2>&1
