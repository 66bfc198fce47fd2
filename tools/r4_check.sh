#!/bin/bash
# Round-4 quick check: GPU tests, smoke, the default bench line, the LDS alignment probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/r4/gputests.log 2>&1 && echo "tests ok" && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4/bench.json 2> gpurun_out/r4/bench.err && echo "bench ok" && \
timeout -k 10 60 ./tools/micro/ulds > gpurun_out/r4/ulds.log 2>&1 && echo "ulds ok" && \
{ [ -z "$AB_LIBS" ] || { bash tools/ab_multi.sh "$AB_LIBS" > gpurun_out/r4/ab.log 2>&1 && echo "ab ok"; }; }
