#!/bin/bash
# the whole GPU suite on the product library, then the headline bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/gputests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/gputests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path --no-secondary --steps 30 > gpurun_out/bench_h.log 2>&1
echo "bench rc=$?"
