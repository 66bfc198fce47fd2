#!/bin/bash
# Round-4: encoder / compaction / decoder times against the number of 256-stream
# workgroups per CU (64, 48, 32, 16 buffers of 4 MiB x 4096 streams: 4, 3, 2, 1
# encoder workgroups per CU), to price a split encode whose halves overlap the
# other half's compaction
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/occ
mkdir -p $O
for B in 64 48 32 16; do
  timeout -k 10 120 python3 bench.py --buffers $B --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-secondary > $O/b$B.json 2> $O/b$B.err || { echo "B=$B failed"; exit 1; }
  echo "B=$B $(python3 -c "import json;d=json.load(open('$O/b$B.json'));print(d['ms_per_step'],d['kernels_ms'],d['roofline']['avg_launch_ms'])")"
done
