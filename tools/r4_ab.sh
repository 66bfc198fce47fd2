#!/bin/bash
# Round-4: GPU tests, the default bench line, a same-box A/B of ab/ libraries
# ($AB_LIBS), the same over the blob workload ($AB_BLOB_LIBS), then the decoder's ablations on the diagnostic build ($DEC_ABLS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/r4/gputests.log 2>&1 && echo "tests ok" && \
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4/bench.json 2> gpurun_out/r4/bench.err && echo "bench ok" && \
{ [ -z "$AB_LIBS" ] || { timeout -k 10 600 bash tools/ab_multi.sh "$AB_LIBS" > gpurun_out/r4/ab.log 2>&1 && echo "ab ok"; }; } && \
{ [ -z "$AB_BLOB_LIBS" ] || { timeout -k 10 600 bash tools/ab_multi.sh "$AB_BLOB_LIBS" --workload blob > gpurun_out/r4/ab_blob.log 2>&1 && echo "ab blob ok"; }; } && \
{ [ -z "$DEC_ABLS" ] || { DEC_ABLS="$DEC_ABLS" timeout -k 10 400 bash tools/dec_ablate.sh > gpurun_out/r4/dec_abl.log 2>&1 && echo "dec abl ok"; }; }
