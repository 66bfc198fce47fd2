#!/bin/bash
# Same-box A/B of the xN encoder's workgroup width (256: 4 table copies, 4
# workgroups per CU; 512: 8 copies, 2 per CU; 1024: 16 copies, one per CU),
# whole step; extra: "<lib> <width>" pairs run through ZR_LIB_PATH
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
B="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-secondary"
for r in $(seq 1 ${ROUNDS:-4}); do
  for w in ${WIDTHS:-256 512 1024}; do
    timeout -k 10 120 $B --enc-width $w > gpurun_out/ab/run.log 2>&1 || { cat gpurun_out/ab/run.log; exit 1; }
    echo "w$w : $(tail -1 gpurun_out/ab/run.log)"
  done
  if [ -n "$EXTRA" ]; then
    set -- $EXTRA
    while [ $# -ge 2 ]; do
      ZR_LIB_PATH=$1 timeout -k 10 120 $B --enc-width $2 > gpurun_out/ab/run.log 2>&1 || { cat gpurun_out/ab/run.log; exit 1; }
      echo "$(basename $1)_w$2 : $(tail -1 gpurun_out/ab/run.log)"
      shift 2
    done
  fi
done
