set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr_lv -o lv -- python3 bench.py --steps 1 --warmup 0 --no-bfs --no-traffic --no-cpu-baseline --louvain-scale ${LS:-23} > gpurun_out/tr_lv.log 2>&1; rc=$?
grep "\[bench\]" gpurun_out/tr_lv.log; python3 scripts/trace_gaps.py /tmp/tr_lv; exit $rc
