# rocprofv3 PMC passes (one counter group per pass, each under its own time limit)
# over one bench child (graph build + one algorithm call).
# usage: TAG=x WHAT=pagerank|bfs SCALE=24 bash scripts/gpu_pmc.sh "GROUP1" "GROUP2" ...
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-pmc}; WHAT=${WHAT:-pagerank}; SCALE=${SCALE:-24}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$WHAT" = bfs ]; then CHILD="--traffic-child bfs --bfs-scale $SCALE --bfs-roots 8"; else CHILD="--traffic-child pagerank --scale $SCALE"; fi
i=0
for grp in "$@"; do
  i=$((i+1))
  rm -rf /tmp/pmc_$i
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_$i -o pmc -- python3 bench.py $CHILD > $OUT/pass$i.log 2>&1
  rc=$?
  f=$(find /tmp/pmc_$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && cp "$f" $OUT/pass$i.csv
  echo "pass $i ($grp): rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
