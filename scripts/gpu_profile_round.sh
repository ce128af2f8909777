# Round profile: kernel-trace stats of the default bench (PageRank + BFS + Louvain legs)
# and the bench line itself (which runs its own PMC traffic passes).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; grep "\[bench\]" $OUT/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_round -o bench -- python3 bench.py --no-traffic --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?
f=$(find /tmp/prof_round -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv; exit $rc
