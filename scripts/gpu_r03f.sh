#!/bin/bash
# round 3 step f: MG tests (world-8 Louvain hang check) + push SQ counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_mg.log 2>&1; rc=$?
tail -3 $O/pytest_mg.log; grep -E "FAILED|Timeout|Fatal Python" $O/pytest_mg.log | head
[ $rc -eq 0 ] || exit $rc
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM" \
           "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA"; do
  i=$((i+1)); rm -rf /tmp/pmc$i
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc$i -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/pr_ab.py 24 base > $GRAFT_REPO_ROOT/$O/pmc$i.log 2>&1) || { echo "pmc $i failed"; tail -5 $O/pmc$i.log; exit 1; }
  python3 scripts/pmc_push.py /tmp/pmc$i >> $O/pmc.txt
  echo "pmc set $i done"
done
cat $O/pmc.txt
echo ALLDONE
