#!/bin/bash
# PMC A/B of two library builds on one box: pmc_ab.sh <libA> <libB> <kernel-regex> [bench args]
# (SQ issue/wait counters, then FETCH_SIZE and WRITE_SIZE, each its own pass)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=$1; Bl=$2; K=$3; shift 3
O=gpurun_out/pmcab
mkdir -p $O
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path $*"
for L in $A $Bl; do
  t=$(basename $L .so)
  export ZR_LIB_PATH=$PWD/$L
  timeout -k 10 120 rocprofv3 --kernel-include-regex "$K" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O -o ${t}_sq -- $B > $O/${t}_sq.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE --output-format csv -d $O -o ${t}_f -- $B > $O/${t}_f.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-include-regex "$K" --pmc WRITE_SIZE --output-format csv -d $O -o ${t}_w -- $B > $O/${t}_w.log 2>&1
done
python3 tools/pmc_sum.py $O/*_counter_collection.csv > $O/sum.txt
