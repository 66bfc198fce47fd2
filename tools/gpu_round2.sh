set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests -m gpu > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/b_rans.log 2>&1 && \
timeout -k 10 300 python3 bench.py --buffers 1 --buffer-mib 256 --steps 4 > gpurun_out/b_lit.log 2>&1 && \
timeout -k 10 300 bash tools/ab_lib.sh zipora_amd/ab/lib_HEAD.so zipora_amd/libzipora_amd.so > gpurun_out/ab1.log 2>&1 && \
timeout -k 10 300 bash tools/trace_step.sh > /dev/null 2>&1
