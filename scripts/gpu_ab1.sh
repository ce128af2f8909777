set -o pipefail
MODES="16" bash scripts/ablate.sh 2>&1 | tee gpurun_out/ablate16.log &&
LIBS="cugraph-forked_amd/lib/libcugraph_c.so scripts/variants/w14.so scripts/variants/w14p16.so scripts/variants/t512p16.so" STEPS=10 EXTRA="--epsilon 1e9" bash scripts/ab.sh 2>&1 | tee gpurun_out/ab1.log
