#!/bin/bash
# Snapshot the CURRENT working tree's extension as build/ab/<NAME>/_C.so (for one-box A/B runs
# of uncommitted kernel variants:  MINGPT_EXT_SO=build/ab/<NAME>/_C.so python bench.py).
set -e
cd "$(dirname "$0")/.."
NAME=$1
D=/tmp/var_$NAME
rm -rf "$D" && mkdir -p "$D"
cp -r csrc build_ext.py "$D/" && mkdir -p "$D/mingpt_distributed_amd"
# MG_PATCH=<file>: apply a diagnostic patch to the scratch copy only (e.g. bench/dev/attn_ablations.patch
# + MG_EXTRA_FLAGS=-DMG_ABL_NOEXP: the timing-only attention ablations, outputs wrong on purpose)
if [ -n "$MG_PATCH" ]; then (cd "$D" && patch -p1 < "$OLDPWD/$MG_PATCH" >/dev/null); fi
python "$D/build_ext.py" >/dev/null
mkdir -p "build/ab/$NAME" && cp "$D/mingpt_distributed_amd/_C.so" "build/ab/$NAME/_C.so"
echo "build/ab/$NAME/_C.so"
