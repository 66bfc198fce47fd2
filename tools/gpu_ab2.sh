set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
true && \
timeout -k 10 400 bash tools/ab_lib.sh zipora_amd/ab/lib_HEAD.so zipora_amd/libzipora_amd.so > gpurun_out/ab1.log 2>&1 && \
timeout -k 10 400 bash tools/ab_lib.sh zipora_amd/ab/lib_HEAD.so zipora_amd/libzipora_amd.so --buffers 1 --buffer-mib 256 --steps 4 >> gpurun_out/ab1.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-host-path > gpurun_out/b1.log 2>&1 && \
timeout -k 10 300 bash tools/trace_step.sh > /dev/null 2>&1
