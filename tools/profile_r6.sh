#!/bin/bash
# Round-6 profile (round 5 recipe): kernel-trace stats of every bench workload, PMC traffic
# (FETCH_SIZE and WRITE_SIZE in separate passes), SQ counters, and the default
# bench command under a kernel trace (its JSON line + the timed region).
set -o pipefail
R=${1:-r06}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_$R
mkdir -p $O/summary
B="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-secondary"
L="python3 bench.py --buffers 1 --buffer-mib 256 --no-cpu-baseline --no-host-path --no-secondary"
N18="python3 bench.py --buffers 1 --buffer-mib 256 --streams 262144 --no-cpu-baseline --no-host-path --no-secondary"
run() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
run trace_rans timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rans -o rans -- $B > $O/rans_bench.log 2>&1
run trace_lit timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lit -o lit -- $L --steps 3 --warmup 1 > $O/lit_bench.log 2>&1
run trace_n18 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n18 -o n18 -- $N18 --steps 10 --warmup 3 > $O/n18_bench.log 2>&1
run trace_fse timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fse -o fse -- python3 bench.py --workload fse --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $O/fse_bench.log 2>&1
run trace_o1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/o1 -o o1 -- python3 bench.py --workload o1 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/o1_bench.log 2>&1
run trace_blob timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/blob -o blob -- python3 bench.py --workload blob --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary > $O/blob_bench.log 2>&1
for f in $(find $O -name "*kernel_stats.csv"); do cp $f $O/summary/; done
K="--kernel-include-regex k_dec_xn_fast|k_enc_xn|k_enc_compact|k_hist|k_fse_dec|k_fse_enc|k_copy16|k_enc_x1_fast|k_enc_x1_ring|k_dec_x1_fast|k_dec_x1_ring|k_hist_small"
BP="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary"
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  run pmc_$n timeout -s KILL 90 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_$n -o $n -- $BP > $O/pmc_$n.log 2>&1
  run pmc_lit_$n timeout -s KILL 90 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_lit_$n -o $n -- $L --steps 1 --warmup 1 > $O/pmc_lit_$n.log 2>&1
  run pmc_n18_$n timeout -s KILL 90 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_n18_$n -o $n -- $N18 --steps 1 --warmup 1 > $O/pmc_n18_$n.log 2>&1
  run pmc_fse_$n timeout -s KILL 120 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_fse_$n -o $n -- python3 bench.py --workload fse --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $O/pmc_fse_$n.log 2>&1
  run pmc_blob_$n timeout -s KILL 120 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_blob_$n -o $n -- python3 bench.py --workload blob --steps 1 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary > $O/pmc_blob_$n.log 2>&1
  run pmc_o1_$n timeout -s KILL 90 rocprofv3 $K --pmc $c --output-format csv -d $O/pmc_o1_$n -o $n -- python3 bench.py --workload o1 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $O/pmc_o1_$n.log 2>&1
done
run sq1 timeout -s KILL 90 rocprofv3 $K --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/sq1 -o sq1 -- $BP > $O/sq1.log 2>&1
run sq2 timeout -s KILL 90 rocprofv3 $K --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o sq2 -- $BP > $O/sq2.log 2>&1
python3 tools/pmc_sum.py $(find $O/sq1 $O/sq2 -name "*counter_collection.csv") > $O/summary/sq_counters.txt 2>&1 || true
run bench_trace timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bc -o bc -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/summary/bench.json 2> $O/bench_cmd.err
python3 tools/timed_region.py $(find $O/bc -name "*kernel_trace.csv" | head -1) 5 20 > $O/summary/bench_cmd_timed_region.txt
cp $(find $O/bc -name "*kernel_stats.csv" | head -1) $O/summary/bench_cmd_kernel_stats.csv
echo "profile done"
