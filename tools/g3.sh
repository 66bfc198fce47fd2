set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/gputests.log 2>&1
echo "gputests rc=$?"
tail -3 gpurun_out/gputests.log
timeout -k 10 400 bash tools/ab_multi.sh "zipora_amd/ab/lib_base.so zipora_amd/ab/lib_new.so" > gpurun_out/ab3.log 2>&1
echo "ab rc=$?"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err
echo "bench rc=$?"
