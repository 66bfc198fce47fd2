#!/bin/bash
# clocks and power while the headline step runs back to back (is the step power-limited?)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 bench.py --steps 12000 --warmup 5 --no-cpu-baseline --no-host-path > gpurun_out/power_bench.log 2>&1 &
B=$!
sleep 12
for i in 1 2 3 4 5 6; do timeout 20 rocm-smi --showpower --showclocks --showtemp >> gpurun_out/power.log 2>&1; sleep 0.5; done
wait $B
echo "bench rc=$?" >> gpurun_out/power.log
timeout 20 rocm-smi --showpower --showclocks --showtemp >> gpurun_out/power_idle.log 2>&1
exit 0
