#!/bin/bash
# Round-4: host pipeline with 3 device slots (ab/lib_slots3.so) against 2 (ab/lib_slots2.so), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pipe
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARS:-slots2 slots3}; do
    ZR_LIB_PATH=zipora_amd/ab/lib_$v.so timeout -k 10 200 python3 tools/pipe_ab.py > $O/${v}_$r.log 2>&1 || { tail -5 $O/${v}_$r.log; exit 1; }
    sed "s/^/$v r$r /" $O/${v}_$r.log
  done
done
