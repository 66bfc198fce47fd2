#!/bin/bash
# Round-6 close: the driver's checks (GPU tests, smoke, torchrun headline), then
# tools/profile_r6.sh (kernel stats of every workload, PMC traffic, SQ counters,
# the default bench command under a kernel trace) into gpurun_out/prof_$1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/final_check.sh && echo "final checks ok" && \
bash tools/profile_r6.sh ${1:-r06z} > gpurun_out/profile_${1:-r06z}.log 2>&1 && echo "profile ok"
