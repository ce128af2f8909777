#!/bin/bash
# round 3: MG Louvain / BFS tests, BFS bench + per-traversal timeline, memory calibration
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_bfs.py tests/test_gpu_bench_parity.py tests/test_gpu_louvain.py -m gpu -x -v --timeout 300 --timeout-method thread --durations=20 > $O/pytest.log 2>&1 || { echo pytest failed; exit 1; }
timeout -k 10 300 python -u bench.py --bfs-only --no-cpu-baseline > $O/bfs.json 2> $O/bfs.err || { echo bfs failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr_bfs -o tr -- python3 bench.py --bfs-only --no-cpu-baseline --bfs-reps 2 > $O/bfs_tr.log 2>&1 || { echo trace failed; exit 1; }
python3 scripts/bfs_timeline.py /tmp/tr_bfs 3 > $O/bfs_timeline.txt 2>&1
timeout -k 10 400 bash scripts/gpu_calib.sh || { echo calib failed; exit 1; }
echo ALLDONE
