set -o pipefail
CGX_BFS_DEBUG=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-louvain --no-traffic --bfs-roots 2 > gpurun_out/bfs_levels.log 2>&1; rc=$?
grep "\[bfs\]\|\[bench\] bfs" gpurun_out/bfs_levels.log | tail -24; exit $rc
