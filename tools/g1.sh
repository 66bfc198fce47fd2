set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_rans.log 2>&1 && \
timeout -k 10 400 bash tools/dec_ablate.sh > gpurun_out/dec_ablate.log 2>&1
