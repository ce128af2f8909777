#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then separate PMC passes.
# usage: scripts/profile.sh <tag> [bench args...]
set -u
TAG=${1:-run}; shift || true
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="${@:---no-bfs --no-cpu-baseline --no-traffic --steps 3 --warmup 1}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 "$ROOT/bench.py" $ARGS > "$OUT/kt.log" 2>&1 || { echo "kt failed"; tail -20 "$OUT/kt.log"; exit 1; }
echo "kernel trace done"
if [ -n "${PMC_SETS:-}" ]; then
  i=0
  for set in $PMC_SETS; do
    i=$((i+1))
    ctrs=$(echo "$set" | tr ',' ' ')
    timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/pmc$i" -o pmc -- python3 "$ROOT/bench.py" $ARGS > "$OUT/pmc$i.log" 2>&1 || { echo "pmc $i failed"; tail -20 "$OUT/pmc$i.log"; exit 1; }
    echo "pmc set $i ($set) done"
  done
fi
find "$OUT" -name "*stats*.csv" | head
