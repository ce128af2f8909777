#!/bin/bash
# round 3 step c: BFS tests + probe-grid A/B, PageRank gather ablation, new tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py::test_unit_weights_take_unweighted_push -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in - CGX_BFS_PROBE_GRID=2048 CGX_BFS_PROBE_GRID=4096 CGX_BFS_PROBE_GRID=8192,CGX_BFS_RES_GRID=4096 CGX_BFS_RES_GRID=4096 CGX_BFS_NO_SPEC=1; do
  envs=""; [ "$m" = "-" ] || envs="${m//,/ }"
  env $envs timeout -k 10 200 python -u bench.py --bfs-only --no-cpu-baseline --bfs-reps 3 > $O/bfs_$m.json 2> $O/bfs_$m.err || { tail $O/bfs_$m.err; exit 1; }
  echo "== $m: $(grep '\[bench\]' $O/bfs_$m.err)"
done
timeout -k 10 300 python -u scripts/pr_ab.py 24 base CGX_PR_ABLATE_XMASK=0xFFFF CGX_PR_ABLATE_XMASK=0x3FFFF CGX_PR_ABLATE_XMASK=0xFFFFF CGX_PR_ABLATE_XMASK=0x3FFFFF base > $O/pr_ab.txt 2>&1 || { tail $O/pr_ab.txt; exit 1; }
cat $O/pr_ab.txt
echo ALLDONE
