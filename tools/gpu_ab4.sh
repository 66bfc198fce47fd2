set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 bash tools/ab_lib.sh zipora_amd/ab/lib_HEAD.so zipora_amd/ab/lib_dec_nt.so > gpurun_out/ab1.log 2>&1 && \
timeout -k 10 300 bash tools/ab_lib.sh zipora_amd/ab/lib_HEAD.so zipora_amd/ab/lib_cmp_nt.so >> gpurun_out/ab1.log 2>&1
