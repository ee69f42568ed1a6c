#!/bin/bash
# Snapshot git revision REV as a runnable tree under build/ab/tree_<sha>/ (package + its built _C.so +
# bench.py), for one-box A/Bs of changes that touch both Python and kernels:
#   python build/ab/tree_<sha>/bench.py ...      (bench.py puts its own directory first on sys.path)
# The revision is exported with `git archive` into a fresh temporary directory (no worktree
# registrations left in .git, no stale checkout reused) that is removed afterwards.
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
SHA=$(git rev-parse --short "$REV")
WT=$(mktemp -d /tmp/ab_src_XXXXXX)
trap 'rm -rf "$WT"' EXIT
git archive "$SHA" | tar -x -C "$WT"
python "$WT/build_ext.py" >/dev/null
DST=build/ab/tree_$SHA
rm -rf "$DST" && mkdir -p "$DST"
cp -r "$WT/mingpt_distributed_amd" "$WT/bench.py" "$DST/"
find "$DST" -name __pycache__ -prune -exec rm -rf {} +
echo "$DST"
