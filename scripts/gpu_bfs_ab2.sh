set -o pipefail
run() { CUGRAPH_AMD_LIB=$2 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-louvain --no-traffic --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["bfs"]; print(sys.argv[1], round(d["mteps_harmonic_mean"]), round(d["ms_mean"],3))' $1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_bfs.py tests/test_gpu_mg.py -k "bfs or path" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_bfs.log 2>&1; rc=$?; tail -2 gpurun_out/pt_bfs.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  run p8bf cugraph-forked_amd/lib/libcugraph_c.so || exit 1
  run p8 scripts/variants/p8.so || exit 1
done
