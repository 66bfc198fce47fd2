#!/bin/bash
# decoder ablations of the wide kernel (diag build), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DEC_ABLS="${DEC_ABLS:-0 64 128 192 256 1 4}" timeout -k 10 500 bash tools/dec_ablate.sh > gpurun_out/dec_abl3.log 2>&1
echo "abl rc=$?"
