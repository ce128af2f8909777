set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/b.log 2> gpurun_out/b.err; rc=$?; grep "\[bench\]" gpurun_out/b.err
tail -1 gpurun_out/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("PR", d["value"], d["ms_per_step"], d["roofline"]["avg_kernel_ms"]); print("BFS", d["bfs"]["mteps_harmonic_mean"], d["bfs"]["ms_mean"])'
exit $rc
