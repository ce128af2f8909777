#!/bin/bash
# One GPU call: SSSP parity tests, the SSSP bench leg, and a kernel trace of it.
# usage: TAG=r06c bash scripts/gpu_sssp.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-sssp}
mkdir -p $OUT
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sssp.py -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -8 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --sssp-only ${BENCH_ARGS:-} > $OUT/sssp.json 2> $OUT/sssp.err
rc=$?; grep "\[bench\]" $OUT/sssp.err; [ $rc -eq 0 ] || { tail -20 $OUT/sssp.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_sssp -o sssp -- python3 bench.py --sssp-only --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
rc=$?
for f in $(find /tmp/prof_sssp -name "*kernel_stats.csv" -o -name "*kernel_trace.csv"); do cp "$f" $OUT/; done
exit $rc
