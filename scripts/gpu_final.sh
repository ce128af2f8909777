set -o pipefail
bash scripts/gpu_suite.sh || exit 1
start=$(date +%s)
timeout -k 10 600 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err; rc=$?
echo "bench rc=$rc wall=$(( $(date +%s) - start ))s"
tail -1 gpurun_out/final_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['metric'], d['value'], d['unit'], d['ms_per_step'], round(d['roofline']['frac'],4), d['roofline']['traffic'], d['cpu_baseline']['value'], d['bfs']['mteps_harmonic_mean'], d['louvain']['time_s'])"
exit $rc
