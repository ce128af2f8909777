set -o pipefail
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-louvain --no-traffic"
for rep in 1 2; do
for cfg in "40 24" "40 64" "80 64" "150 64" "80 128"; do
  set -- $cfg
  CGX_BFS_ALPHA=$1 CGX_BFS_BETA=$2 timeout -k 10 200 $B > gpurun_out/bfs_ab.json 2>/dev/null || exit 1
  tail -1 gpurun_out/bfs_ab.json | python -c "import json,sys; d=json.loads(sys.stdin.read())['bfs']; print('a=$1 b=$2', round(d['mteps_harmonic_mean']), round(d['ms_mean'],3))"
done
done
