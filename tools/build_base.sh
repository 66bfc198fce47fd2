#!/bin/bash
# Builds the library of a git revision (default HEAD) into zipora_amd/ab/lib_<rev>.so
# for same-box A/B runs (tools/ab_lib.sh). Run here, not on the GPU box.
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" worktree add -q --detach "$T" "$REV"
(cd "$T" && python3 -m zipora_amd.build >/dev/null)
mkdir -p "$ROOT/zipora_amd/ab"
cp "$T/zipora_amd/libzipora_amd.so" "$ROOT/zipora_amd/ab/lib_$REV.so"
git -C "$ROOT" worktree remove --force "$T"
echo "$ROOT/zipora_amd/ab/lib_$REV.so"
