set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 500 bash tools/ab_multi.sh "zipora_amd/ab/lib_HEAD.so zipora_amd/ab/lib_cur.so" --workload fse --steps 5 > gpurun_out/ab1.log 2>&1
