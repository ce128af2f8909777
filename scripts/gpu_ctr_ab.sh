set -o pipefail
S="TCC_HIT_sum,TCC_MISS_sum TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_DRAM_sum TCC_ATOMIC_sum,TCC_EA0_ATOMIC_sum FETCH_SIZE WRITE_SIZE"
SETS="$S" TAG=queue timeout -k 10 400 bash scripts/gpu_counters.sh > gpurun_out/ctr_queue.txt 2>&1
CGX_PR_PUSH=static SETS="$S" TAG=static timeout -k 10 400 bash scripts/gpu_counters.sh > gpurun_out/ctr_static.txt 2>&1
grep -v "^set" gpurun_out/ctr_queue.txt; echo ----; grep -v "^set" gpurun_out/ctr_static.txt
