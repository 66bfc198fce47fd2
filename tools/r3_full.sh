#!/bin/bash
# the driver's sequence: GPU tests, smoke, default bench (all lines), plus the headline's kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
echo "rc=$?"
