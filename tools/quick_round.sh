#!/bin/bash
# GPU tests, smoke and the headline + literal bench lines (logs under gpurun_out/)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/bench_rans.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/bench_rans2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --buffers 1 --buffer-mib 256 --steps 4 --no-cpu-baseline --no-host-path > gpurun_out/bench_lit.log 2>&1
