# BFS leg (RMAT-24, 8 roots) under handle options, one bench child each
# usage: TAG=x bash scripts/bfs_opts_ab.sh "opt1=v" "opt2=v,opt3=v" ...
set -o pipefail
OUT=gpurun_out/${TAG:-bfsopt}; mkdir -p $OUT
i=0
for o in "" "$@" ""; do
  i=$((i+1))
  timeout -k 10 240 python -u bench.py --bfs-only --no-traffic --no-cpu-baseline --options "$o" > $OUT/r$i.json 2> $OUT/r$i.err || exit 1
  python -c "import json; d=json.load(open('$OUT/r$i.json')); print('[$o]', round(d['ms_mean'],4), [round(x,3) for x in d['ms_per_root_median']])"
done
