#!/bin/bash
# GPU tests on the in-tree library, then a same-box headline A/B of the given libraries
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 500 bash tools/ab_multi.sh "$1" > gpurun_out/abr.log 2>&1 && \
timeout -k 10 500 bash tools/ab_multi.sh "$1" >> gpurun_out/abr.log 2>&1
