set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tenc
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o t -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/b.log 2>&1
python3 tools/kdur.py $(find $O -name "*kernel_trace.csv" | head -1) k_enc_xn > $O/enc.txt
python3 tools/kdur.py $(find $O -name "*kernel_trace.csv" | head -1) k_dec_xn_fast > $O/dec.txt
