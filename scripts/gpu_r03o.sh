#!/bin/bash
# world-8 Louvain rehearsal with HSA_ENABLE_SDMA=0 in the ranks (tests/test_gpu_mg.py
# _rank_setup), five runs, each a fresh pytest under the test's own 150 s deadline;
# stops at the first failure
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03o
timeout -k 10 1000 python - <<'PY'
import subprocess, sys, time
for i in range(5):
    t = time.time()
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "tests/test_gpu_mg.py", "-q", "-x",
                        "--timeout", "200", "--timeout-method", "thread", "-k", "world8 and louvain"],
                       capture_output=True, text=True, timeout=190)
    line = [l for l in r.stdout.splitlines() if "passed" in l or "failed" in l]
    print(f"run {i}: rc {r.returncode} {time.time() - t:.1f}s {line[-1] if line else ''}", flush=True)
    open(f"gpurun_out/r03o/w8_{i}.log", "w").write(r.stdout + r.stderr)
    if r.returncode != 0:
        sys.exit(1)
PY
