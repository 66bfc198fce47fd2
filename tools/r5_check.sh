#!/bin/bash
# Round 5 check: the whole GPU suite, smoke, then the default bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_tests_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_tests_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r5_bench_default.json 2> gpurun_out/r5_bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r5_bench_default.json
