#!/bin/bash
# Builds the current working tree's library into zipora_amd/ab/lib_<name>.so
# (for same-box A/B of uncommitted variants), optionally after a python patch
# script run on the copy (argv[1] = the copy's root). Run here, not on the GPU box.
#   tools/build_wt.sh <name> [patch.py]
set -e
NAME=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p "$T/zipora_amd" "$T/include"
cp -r "$ROOT/zipora_amd/csrc" "$ROOT/zipora_amd/build.py" "$T/zipora_amd/"
cp "$ROOT/include/"*.h "$T/include/"
if [ -n "$2" ]; then python3 "$2" "$T"; fi
(cd "$T" && python3 zipora_amd/build.py >/dev/null)
mkdir -p "$ROOT/zipora_amd/ab"
cp "$T/zipora_amd/libzipora_amd.so" "$ROOT/zipora_amd/ab/lib_$NAME.so"
rm -rf "$T"
echo "$ROOT/zipora_amd/ab/lib_$NAME.so"
