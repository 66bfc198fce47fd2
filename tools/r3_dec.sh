#!/bin/bash
# fast-path tests, then the headline bench line (no CPU legs), then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fastpath_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/fastpath.log 2>&1
echo "fastpath rc=$?"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path --steps 20 --warmup 5 > gpurun_out/bench_h.log 2> gpurun_out/bench_h.err && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/gputests.log 2>&1
echo "rc=$?"
