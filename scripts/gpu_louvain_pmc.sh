#!/bin/bash
# PMC counters of the Louvain local-move kernels (bench.py --louvain-only, RMAT-23):
# one rocprofv3 --pmc pass per counter group, per-kernel averages (scripts/pmc_kernels.py).
# usage: TAG=r05e bash scripts/gpu_louvain_pmc.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-lvpmc}; mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" "SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM"; do
  i=$((i+1)); d=/tmp/lvpmc_$i; rm -rf $d
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $d -o run --output-format csv -- python3 bench.py --louvain-only > $OUT/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pass$i.log; exit 1; }
  f=$(find $d -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_kernels.py "$f" k_big_partials k_big_buckets k_sweep_hash k_vertex_weights radix_sort_onesweep >> $OUT/pmc.txt
done
cat $OUT/pmc.txt
