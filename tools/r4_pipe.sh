#!/bin/bash
# Round-4: same-box A/B of the headline step: serial vs --pipeline, 256 vs 1024 encoder
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
for r in 1 2 3; do
  for V in "" "--pipeline" "--enc-width 1024" "--pipeline --enc-width 1024"; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-secondary $V \
      > gpurun_out/r4/pipe_run.json 2> gpurun_out/r4/pipe_run.err || { tail -5 gpurun_out/r4/pipe_run.err; exit 1; }
    python3 - "$V" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r4/pipe_run.json").read().strip().splitlines()[-1])
print(f"[{sys.argv[1]:28s}] value {d['value']:8.2f} ms/step {d['ms_per_step']:.4f} kernels {d['kernels_ms']} timed enc {d['roofline']['avg_launch_ms']} dec {d['roofline_decode']['avg_launch_ms']}")
PY
  done
done
