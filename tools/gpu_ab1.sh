set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_rans_r02_gpu.py tests/test_rans_gpu.py tests/test_kats_r02.py tests/test_compressor.py -m gpu > gpurun_out/t1.log 2>&1 && \
timeout -k 10 400 bash tools/ab_lib.sh zipora_amd/ab/lib_HEAD.so zipora_amd/libzipora_amd.so > gpurun_out/ab1.log 2>&1 && \
timeout -k 10 400 bash tools/ab_lib.sh zipora_amd/ab/lib_HEAD.so zipora_amd/libzipora_amd.so --buffers 1 --buffer-mib 256 --steps 4 >> gpurun_out/ab1.log 2>&1
