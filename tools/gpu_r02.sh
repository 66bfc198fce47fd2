#!/bin/bash
# Round-2 GPU check: new parity tests first, then the whole -m gpu suite,
# smoke, and the headline + literal configs[1] bench lines (logs in gpurun_out/).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 170 --timeout-method thread"
timeout -k 10 400 $T tests/test_rans_r02_gpu.py tests/test_kats_r02.py -m gpu > gpurun_out/r02_new.log 2>&1 && \
timeout -k 10 600 $T tests -m gpu > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_rans.log 2>&1 && \
timeout -k 10 300 python -u bench.py --buffers 1 --buffer-mib 256 > gpurun_out/bench_lit.log 2>&1
