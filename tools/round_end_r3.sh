#!/bin/bash
# Round-3 close: the driver's checks (GPU tests, smoke, torchrun headline),
# kernel-trace stats and PMC passes of every workload (profile_r3a/b), the
# default bench under a kernel trace (its JSON line + the timed region's
# per-dispatch durations), then a same-box A/B of ab/ libraries ($AB_LIBS)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_r03
mkdir -p $O/summary
bash tools/final_check.sh && echo "final checks ok" && \
bash tools/profile_r3a.sh r03 > $O/r3a.log 2>&1 && echo "profile A ok" && \
bash tools/profile_r3b.sh r03 > $O/r3b.log 2>&1 && echo "profile B ok" && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bc -o bc -- python3 bench.py > $O/summary/bench.json 2> $O/bench_cmd.err && \
python3 tools/timed_region.py $(find $O/bc -name "*kernel_trace.csv" | head -1) > $O/summary/bench_cmd_timed_region.txt && \
cp $(find $O/bc -name "*kernel_stats.csv" | head -1) $O/summary/bench_cmd_kernel_stats.csv && echo "bench trace ok" && \
{ [ -z "$AB_LIBS" ] || bash tools/ab_multi.sh "$AB_LIBS"; }
