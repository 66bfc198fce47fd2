#!/bin/bash
# Round-3 profile, part A: kernel-trace stats of every bench workload (rocprofv3 --kernel-trace --stats).
set -e
R=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_$R
mkdir -p $O/summary
B="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-secondary"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rans -o rans -- $B > $O/rans_bench.log 2>&1
L="python3 bench.py --buffers 1 --buffer-mib 256 --no-cpu-baseline --no-host-path --no-secondary"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lit -o lit -- $L --steps 3 --warmup 1 > $O/lit_bench.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fse -o fse -- python3 bench.py --workload fse --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $O/fse_bench.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/o1 -o o1 -- python3 bench.py --workload o1 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/o1_bench.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/blob -o blob -- python3 bench.py --workload blob --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary > $O/blob_bench.log 2>&1
for f in $(find $O -name "*kernel_stats.csv"); do cp $f $O/summary/; done
ls -la $O/summary
