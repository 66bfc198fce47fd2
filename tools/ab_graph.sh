#!/bin/bash
# Round 6: the headline step eager vs HIP-graph replay (bench.py --graph 1), same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/graph
timeout -k 10 300 python -u -m pytest tests/test_graph_capture_gpu.py -x -q --timeout 170 --timeout-method thread > gpurun_out/graph/tests.log 2>&1 || { tail -20 gpurun_out/graph/tests.log; exit 1; }
for r in 1 2 3 4 5; do
  for gmode in 0 1; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-secondary --graph $gmode > gpurun_out/graph/run.log 2>&1 || { cat gpurun_out/graph/run.log; exit 1; }
    echo "graph=$gmode: $(tail -1 gpurun_out/graph/run.log)"
  done
done > gpurun_out/graph/ab.log && echo ok
