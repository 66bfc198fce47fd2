#!/bin/bash
# Round profile: kernel-trace stats for the bench workloads plus the HBM
# traffic PMC passes (FETCH_SIZE and WRITE_SIZE in separate passes, as the
# gfx950 TCC slots require). Run on the GPU box from the repo root:
#   gpurun -- 'bash tools/profile_round.sh r01'
# then copy gpurun_out/prof_<round>/summary/* into profiles/.
set -e
R=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_$R
mkdir -p $O/summary
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path"
BP="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path"
K="--kernel-include-regex k_dec_xn_fast|k_enc_xn|k_enc_compact|k_hist|k_fse_dec|k_fse_enc|k_copy16|k_enc_x1_fast|k_enc_x1_ring|k_dec_x1_fast|k_dec_x1_ring|k_hist_small"
# 1. rANS (headline) kernel trace + stats, default bench command
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rans -o rans -- $B > $O/rans_bench.log 2>&1
# 2. HBM traffic, one counter group per pass
timeout -k 10 300 rocprofv3 $K --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o fetch -- $BP > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o write -- $BP > $O/pmc_write.log 2>&1
# 2a. SQ issue/wait/LDS counters of the headline kernels (8 SQ slots per pass)
timeout -k 10 300 rocprofv3 $K --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/sq1 -o sq1 -- $BP > $O/sq1.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o sq2 -- $BP > $O/sq2.log 2>&1
# 2b. the literal configs[1] (one 256 MiB buffer, 4096 streams): trace + traffic
L="python3 bench.py --buffers 1 --buffer-mib 256 --no-cpu-baseline --no-host-path"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lit -o lit -- $L --steps 3 --warmup 1 > $O/lit_bench.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc FETCH_SIZE --output-format csv -d $O/pmc_lit_fetch -o fetch -- $L --steps 1 --warmup 1 > $O/pmc_lit_fetch.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc WRITE_SIZE --output-format csv -d $O/pmc_lit_write -o write -- $L --steps 1 --warmup 1 > $O/pmc_lit_write.log 2>&1
# 3. FSE workload (configs[2]) kernel trace + stats and traffic
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fse -o fse -- python3 bench.py --workload fse --steps 5 --warmup 2 --no-cpu-baseline > $O/fse_bench.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc FETCH_SIZE --output-format csv -d $O/pmc_fse_fetch -o fetch -- python3 bench.py --workload fse --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fse_fetch.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc WRITE_SIZE --output-format csv -d $O/pmc_fse_write -o write -- python3 bench.py --workload fse --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fse_write.log 2>&1
# 3b. record batch (configs[4]) and O1 shard (configs[3]) traffic
timeout -k 10 300 rocprofv3 $K --pmc FETCH_SIZE --output-format csv -d $O/pmc_blob_fetch -o fetch -- python3 bench.py --workload blob --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > $O/pmc_blob_fetch.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc WRITE_SIZE --output-format csv -d $O/pmc_blob_write -o write -- python3 bench.py --workload blob --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > $O/pmc_blob_write.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc FETCH_SIZE --output-format csv -d $O/pmc_o1_fetch -o fetch -- python3 bench.py --workload o1 --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_o1_fetch.log 2>&1
timeout -k 10 300 rocprofv3 $K --pmc WRITE_SIZE --output-format csv -d $O/pmc_o1_write -o write -- python3 bench.py --workload o1 --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_o1_write.log 2>&1
# 4. O1 shard (configs[3]) and record batch (configs[4]) kernel traces
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/o1 -o o1 -- python3 bench.py --workload o1 --steps 10 --warmup 3 --no-cpu-baseline > $O/o1_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/blob -o blob -- python3 bench.py --workload blob --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > $O/blob_bench.log 2>&1
python3 tools/summarize_prof.py $O > $O/summary/summary.txt 2>&1 || true
python3 tools/pmc_sum.py $(find $O/sq1 $O/sq2 -name "*counter_collection.csv") > $O/summary/sq_counters.txt 2>&1 || true
for f in $(find $O -name "*kernel_stats.csv"); do cp $f $O/summary/; done
ls -la $O/summary
