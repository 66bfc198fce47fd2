#!/bin/bash
# Round-3 GPU check: gpu tests, smoke, default bench line, kernel-trace stats of the headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03a -o rans -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > gpurun_out/prof_r03a.log 2>&1
