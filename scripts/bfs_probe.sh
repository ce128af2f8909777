#!/bin/bash
# BFS check + measurement on the GPU box: parity tests, bench BFS leg, kernel sequence of one BFS.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out/pb
timeout -k 10 400 python -m pytest tests/test_gpu_bfs.py -x -q > gpurun_out/bfs_t.log 2>&1 || { tail -30 gpurun_out/bfs_t.log; exit 1; }
tail -1 gpurun_out/bfs_t.log
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/bfs_b.log 2>/dev/null
python3 -c "
import json; d=json.loads(open('gpurun_out/bfs_b.log').read().strip().splitlines()[-1])['bfs']
print('bfs hm %.0f min %.0f max %.0f ms %.3f' % (d['mteps_harmonic_mean'], d['mteps_min'], d['mteps_max'], d['ms_mean']))"
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/pb/kt_"*
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pb" -o kt -- python3 "$R/scripts/probe_bfs.py" --root-index ${ROOT_INDEX:-1} > "$R/gpurun_out/pb/log" 2>&1
cd "$R" && python3 scripts/probe_bfs.py --summarize gpurun_out/pb/kt_kernel_trace.csv > gpurun_out/pb/seq.txt
