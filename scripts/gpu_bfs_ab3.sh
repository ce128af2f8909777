set -o pipefail
run() { timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-louvain --no-traffic --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["bfs"]; print(sys.argv[1], round(d["mteps_harmonic_mean"]), round(d["ms_mean"],3))' $1; }
for rep in 1 2 3; do
  for c in 256 512 1024 2048; do CGX_BFS_TD_CAP=$c run td$c || exit 1; done
done
