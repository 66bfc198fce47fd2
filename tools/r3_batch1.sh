#!/bin/bash
# spread/stagger A/B, decoder wait ablations, power probe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/r3_ab.sh || exit 1
DEC_ABLS="0 64 192 576 512 256 768" timeout -k 10 500 bash tools/dec_ablate.sh > gpurun_out/dec_abl4.log 2>&1
echo "abl rc=$?"
bash tools/power_probe.sh
