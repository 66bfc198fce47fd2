set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ref_asserts.py tests/test_comm_gpu.py tests/test_huff_sync_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/refasserts.log 2>&1
echo "refasserts rc=$?"
DEC_ABLS="0 5 7 16 32 21 37 1" timeout -k 10 500 bash tools/dec_ablate.sh > gpurun_out/dec_ablate2.log 2>&1
