#!/bin/bash
# headline same-box A/B of library builds, 3 alternating rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 bash tools/ab_multi.sh "$1" > gpurun_out/abr.log 2>&1 && \
timeout -k 10 500 bash tools/ab_multi.sh "$1" >> gpurun_out/abr.log 2>&1
