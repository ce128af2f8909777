# Same-box A/B of two library builds on the bench's BFS leg (RMAT-24, 8 roots):
# ab/libcugraph_c_base.so vs ab/libcugraph_c_new.so, alternated twice.
# usage: TAG=x bash scripts/bfs_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-bfsab}; mkdir -p $OUT
for rep in 1 2; do
  for v in base new; do
    CUGRAPH_AMD_LIB=$PWD/ab/libcugraph_c_$v.so timeout -k 10 300 python -u bench.py --bfs-only --no-traffic --no-cpu-baseline > $OUT/$v$rep.json 2> $OUT/$v$rep.err || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/$v$rep.json')); print('$v$rep', round(d['ms_mean'],4), [round(x,3) for x in d['ms_per_root_median']])"
  done
done
