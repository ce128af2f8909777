set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err; rc=$?; grep "\[bench\]" gpurun_out/bench.err; tail -1 gpurun_out/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
MODES="0 1 2 8 3" bash scripts/ablate.sh 2>&1 | tee gpurun_out/ablate.log
