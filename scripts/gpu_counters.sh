# PMC passes over a short PageRank-only bench (one rocprofv3 run per counter set)
set -u
OUT=gpurun_out/ctr_${TAG:-run}
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for set in ${SETS}; do
  i=$((i+1))
  ctrs=$(echo "$set" | tr ',' ' ')
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$ROOT/$OUT/p$i" -o pmc -- python3 "$ROOT/bench.py" --no-bfs --no-louvain --no-cpu-baseline --no-traffic --steps 2 --warmup 1 --epsilon 1e9 > "$ROOT/$OUT/p$i.log" 2>&1)
  echo "set $i ($set) rc=$?"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, re
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_pr_push" not in k and "k_pr_apply" not in k: continue
        m = re.search(r"(k_pr_\w+)", k)
        agg[m.group(1) if m else k[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v)/len(v):.4g}")
PY
