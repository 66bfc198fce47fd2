#!/bin/bash
# Round 5: SQ counters and HBM traffic of the xN decoders on ONE 256 MiB
# uniform buffer at N = 2^18, 2^19, 2^20 (ring 1: k_dec_xn_fast, 2: k_dec_xn_dma),
# four rocprofv3 --pmc passes per point (each pass within the hardware's limits)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_pmc
mkdir -p $O
K="--kernel-include-regex k_dec_xn"
for N in 262144 524288 1048576; do
  for R in 1 2; do
    BP="python3 bench.py --buffers 1 --buffer-mib 256 --streams $N --dec-ring $R --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-secondary"
    P=$O/n${N}_r${R}
    timeout -s KILL 90 rocprofv3 $K --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d ${P}_sq1 -o sq1 -- $BP > ${P}_sq1.log 2>&1 || exit 1
    timeout -s KILL 90 rocprofv3 $K --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d ${P}_sq2 -o sq2 -- $BP > ${P}_sq2.log 2>&1 || exit 1
    timeout -s KILL 90 rocprofv3 $K --pmc FETCH_SIZE --output-format csv -d ${P}_f -o f -- $BP > ${P}_f.log 2>&1 || exit 1
    timeout -s KILL 90 rocprofv3 $K --pmc WRITE_SIZE --output-format csv -d ${P}_w -o w -- $BP > ${P}_w.log 2>&1 || exit 1
    timeout -s KILL 90 rocprofv3 $K --kernel-trace --stats --output-format csv -d ${P}_kt -o kt -- $BP > ${P}_kt.log 2>&1 || exit 1
    echo "N=$N ring=$R done"
  done
done
python3 tools/pmc_sum.py $(find $O -name "*counter_collection.csv" | sort) > $O/summary.txt 2>&1
echo pmc done
