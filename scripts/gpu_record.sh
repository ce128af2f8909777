#!/bin/bash
# Round record: pytest -m gpu, the default bench line, a rocprofv3 kernel-trace +
# stats profile of the bench (kernel stats + the PageRank launches' durations, so the
# summary can drop the post-convergence no-op launches), each step under its own limit.
# usage: TAG=r04a bash scripts/gpu_record.sh [skip-tests]
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${1:-}" != "skip-tests" ]; then
  CGX_TEST_CLOCK=1 timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread --durations=40 > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log
  # 1 = some test failed (the process itself ended normally): still take the bench
  # record; anything else (fault, abort, time limit) ends the call here
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest.log | head; [ $rc -eq 1 ] || exit $rc; }
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; grep "\[bench\]" $OUT/bench.err; [ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
rm -rf /tmp/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o bench -- python3 bench.py --no-traffic --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?
f=$(find /tmp/prof_$TAG -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/kernel_stats.csv
t=$(find /tmp/prof_$TAG -name "*kernel_trace.csv" | head -1)
[ -n "$t" ] && python3 - "$t" $OUT/pr_launches.csv <<'PY'
import csv, sys
rows = csv.DictReader(open(sys.argv[1]))
with open(sys.argv[2], "w") as f:
    f.write("kernel,start_ns,duration_ns\n")
    for r in rows:
        n = r["Kernel_Name"]
        if "k_pr_push" in n or "k_pr_apply" in n or "k_bu_probe" in n or "k_topdown" in n or "k_finish_pred" in n:
            short = n.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].replace("void ", "").split("::")[-1]
            f.write(f"{short},{r['Start_Timestamp']},{int(r['End_Timestamp']) - int(r['Start_Timestamp'])}\n")
PY
exit $rc
