#!/bin/bash
# FETCH_SIZE calibration for the decoders' refill shapes (tools/micro/fetch_cal.hip)
# and the same counters on the record batch's decoder. Output: gpurun_out/fcal/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fcal
mkdir -p $O
M=tools/micro/fetch_cal
timeout -k 10 60 $M > $O/plain.txt 2>&1 || { echo "micro failed"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o f -- $M > $O/f.log 2>&1 || exit 1
P1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
P2="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum"
timeout -s KILL 60 rocprofv3 --pmc $P1 --output-format csv -d $O/r -o r -- $M > $O/r.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc $P2 --output-format csv -d $O/d -o d -- $M > $O/d.log 2>&1 || exit 1
K="--kernel-include-regex k_dec_x1_fast|k_dec_xn_fast|k_enc_xn|k_hist|k_enc_compact|k_enc_x1_ring"
BL="python3 bench.py --workload blob --steps 1 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary"
BP="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary"
timeout -s KILL 120 rocprofv3 $K --pmc $P1 --output-format csv -d $O/rb -o rb -- $BL > $O/rb.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 $K --pmc $P2 --output-format csv -d $O/db -o db -- $BL > $O/db.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 $K --pmc $P1 --output-format csv -d $O/rh -o rh -- $BP > $O/rh.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 $K --pmc $P2 --output-format csv -d $O/dh -o dh -- $BP > $O/dh.log 2>&1 || exit 1
python3 tools/pmc_sum.py $(find $O -name "*counter_collection.csv") > $O/summary.txt 2>&1
echo done
