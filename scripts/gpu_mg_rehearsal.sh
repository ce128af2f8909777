# Rehearse the N>1 bench path on one GPU: torch.distributed (gloo) communicators, small scales.
set -o pipefail
N=${N:-4}
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus $N --comm torch --steps 2 --warmup 1 --scale ${S:-17} --bfs-scale ${S:-17} --louvain-scale ${S:-17} > gpurun_out/bl_mg.log 2>&1; rc=$?
grep -v Gloo gpurun_out/bl_mg.log | grep "\[bench\]\|Error\|error" | head -20
tail -1 gpurun_out/bl_mg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["parallelism"]); print(d["bfs"]); print(d["louvain"])'
exit $rc
