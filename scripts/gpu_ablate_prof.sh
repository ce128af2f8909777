set -o pipefail
MODES="0 1 2 8 10 4" bash scripts/ablate.sh > gpurun_out/ablate.log 2>&1 && cat gpurun_out/ablate.log &&
PMC_SETS="FETCH_SIZE WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum" bash scripts/profile.sh r01_bfs24 --no-cpu-baseline --no-traffic --steps 1 --warmup 1 --bfs-roots 4
