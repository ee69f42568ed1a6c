#!/bin/bash
# Build the extension of git revision REV (default HEAD) into build/ab/<REV>/_C.so, for one-box
# A/B benches against the working tree:  MINGPT_EXT_SO=build/ab/<REV>/_C.so python bench.py
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
SHA=$(git rev-parse --short "$REV")
WT=/tmp/ab_wt_$SHA
[ -d "$WT" ] || git worktree add -f "$WT" "$SHA" >/dev/null
python "$WT/build_ext.py" >/dev/null
mkdir -p "build/ab/$SHA"
cp "$WT/mingpt_distributed_amd/_C.so" "build/ab/$SHA/_C.so"
echo "build/ab/$SHA/_C.so"
