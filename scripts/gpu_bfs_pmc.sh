# PMC passes over the bench's BFS child (RMAT-24, 8 roots), one counter group per run,
# for the per-dispatch counters of the hub top-down level.
# usage: TAG=x bash scripts/gpu_bfs_pmc.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-bfspmc}; mkdir -p $OUT
i=0
for grp in "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES"; do
  i=$((i+1)); rm -rf /tmp/pmc$i
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc$i -o p -- python3 bench.py --traffic-child bfs --bfs-scale 24 --bfs-roots 8 > $OUT/pass$i.log 2>&1 || exit 1
  f=$(find /tmp/pmc$i -name "*counter_collection.csv" | head -1); gzip -c "$f" > $OUT/pass$i.csv.gz
done
