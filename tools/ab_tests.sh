#!/bin/bash
# GPU tests on the in-tree library, then same-box A/B of the given libraries:
# headline (two alternating rounds) and, with a second argument "blob", the record batch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 500 bash tools/ab_multi.sh "$1" > gpurun_out/abr.log 2>&1 && \
timeout -k 10 500 bash tools/ab_multi.sh "$1" >> gpurun_out/abr.log 2>&1 && \
if [ "$2" = "blob" ]; then timeout -k 10 500 bash tools/ab_multi.sh "$1" --workload blob >> gpurun_out/abr.log 2>&1; fi
