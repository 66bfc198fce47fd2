#!/bin/bash
# Per-dispatch durations of the headline kernels under rocprofv3 --kernel-trace,
# with the bench line of the same run (its roofline.avg_launch_ms must agree
# with the timed-region dispatches of the roofline kernel):
#   gpurun -- 'bash tools/dispatch_trace.sh'   ->  gpurun_out/ddur/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ddur
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o dd -- python3 bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1
T=$(find $O -name "*kernel_trace.csv" | head -1)
for k in k_enc_xn k_dec_xn_fast k_enc_compact_lds k_hist; do echo "== $k"; python3 tools/kdur.py $T $k; done > $O/durations.txt
tail -1 $O/bench.log > $O/bench.json
