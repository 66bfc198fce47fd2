#!/bin/bash
# Decoder ablation timings (diagnostic builds, garbage output): ./dec_abl.sh 0 1 4 5 32 64
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abl; mkdir -p $O
for a in "$@"; do
  ZR_ABLATE=0 ZR_DEC_ABL=$a timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > $O/abl_$a.log 2>&1 || exit 1
  echo "abl $a: $(grep -o '"rans_decode": [0-9.]*' $O/abl_$a.log)"
done
