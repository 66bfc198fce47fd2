#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DEC_ABLS="0 64 192 512 576 256" timeout -k 10 500 bash tools/dec_ablate.sh > gpurun_out/dec_abl5.log 2>&1
echo "abl rc=$?"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path --steps 20 > gpurun_out/bench_h.log 2>&1
echo "bench rc=$?"
