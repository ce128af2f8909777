# Rehearse the N>1 bench path on one GPU: torch.distributed (gloo) communicators, small scales.
# Prints a heartbeat (the log's last [bench] line) every 30 s so a slow rehearsal is not taken as hung.
set -o pipefail
N=${N:-4}
LOG=gpurun_out/bl_mg_$N.log
PYTHONUNBUFFERED=1 timeout -k 10 ${TLIM:-400} python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus $N --comm torch --steps 2 --warmup 1 --scale ${S:-17} --bfs-scale ${S:-17} --louvain-scale ${S:-17} ${EXTRA:-} > $LOG 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do
  sleep 30
  echo "[heartbeat N=$N] $(grep -a '\[bench\]' $LOG | tail -1 | cut -c1-150)"
done
wait $pid; rc=$?
grep -a -v Gloo $LOG | grep -a "\[bench\]\|Error\|error" | head -20
[ $rc -eq 0 ] && tail -1 $LOG | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["parallelism"]); print(d["bfs"]["mteps_harmonic_mean"]); print(d["louvain"])'
exit $rc
