#!/bin/bash
# Round 6: FSE decoder variants, same-box A/B on configs[2] + parity of the variant
#   bash tools/ab_fse.sh "<lib> <lib> ..." <variant lib for parity>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fse
ZR_LIB_PATH=$2 timeout -k 10 300 python -u -m pytest tests/test_fse_gpu.py -x -q --timeout 170 --timeout-method thread > gpurun_out/fse/tests.log 2>&1 && \
ZR_LIB_PATH=$2 timeout -k 10 200 python3 -u tools/fuzz_fse.py 120 ${SEED:-2024} > gpurun_out/fse/fuzz.log 2>&1 && \
for r in $(seq 1 ${ROUNDS:-3}); do
  for L in $1; do
    ZR_LIB_PATH=$L timeout -k 10 200 python3 bench.py --workload fse --steps 5 --warmup 2 --no-cpu-baseline --no-host-path --no-secondary \
      > gpurun_out/fse/run.log 2>&1 || { cat gpurun_out/fse/run.log; exit 1; }
    echo "$(basename $L): $(tail -1 gpurun_out/fse/run.log)"
  done
done > gpurun_out/fse/ab.log && echo ok
