#!/bin/bash
# Alternating A/B of the headline bench: plain vs with the environment setting "$1" (e.g. ZR_DEC_NOFUSE=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/abe_base_$r.log 2>&1 || exit 1
  env $1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/abe_var_$r.log 2>&1 || exit 1
done
