#!/bin/bash
# Kernel trace of the headline step (every kernel, memsets included) -> per-kernel gaps
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/trace
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o step -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path "$@" > $O/step.log 2>&1
python3 tools/gaps.py $(find $O -name "*kernel_trace.csv" | head -1) "k_hist" > $O/gaps.txt
cat $O/gaps.txt
