#!/bin/bash
# Round-4: the split encode (zr_rans_set_encode_split(q)): parity tests, then a
# same-box A/B of the default bench step with --enc-split 0 / 2 / 3 (3 alternations)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/split
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_enc_split_gpu.py tests/test_abi.py -m "gpu or not gpu" -x -q --timeout 170 --timeout-method thread > $O/tests.log 2>&1 && echo "tests ok" || { tail -30 $O/tests.log; exit 1; }
for r in 1 2 3; do
  for sp in ${QS:-0 2 3}; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-secondary --enc-split $sp > $O/b_${sp}_$r.json 2> $O/b_${sp}_$r.err || { cat $O/b_${sp}_$r.err | tail -5; exit 1; }
    echo "split=$sp r=$r $(python3 -c "import json;d=json.load(open('$O/b_${sp}_$r.json'));print(d['value'],d['ms_per_step'],d['kernels_ms'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'])")"
  done
done
