#!/bin/bash
# product-library tests, pair A/B + decoder PMC, grouped-step A/B (ms per step)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export AB_LIBS="zipora_amd/ab/lib_pair0.so zipora_amd/ab/lib_pair1.so"
bash tools/r3_ab.sh || exit 1
for r in 1 2; do for g in 1 2 4; do
  timeout -k 10 120 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-path --no-secondary --groups $g > gpurun_out/grp.log 2>&1 || { cat gpurun_out/grp.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/grp.log').read().strip().splitlines()[-1]); print('groups $g', d['ms_per_step'], d['value'])" >> gpurun_out/groups.log
done; done
bash tools/r3_pmc.sh
