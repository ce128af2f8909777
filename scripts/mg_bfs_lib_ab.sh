# Same-box A/B of two library builds on one-rank MG BFS (scripts/mg_bfs_ab.py):
# ab/libcugraph_c_base.so vs ab/libcugraph_c_new.so, alternated twice.
# usage: TAG=x SCALE=24 bash scripts/mg_bfs_lib_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-mgab}; mkdir -p $OUT
for rep in 1 2; do
  for v in base new; do
    CUGRAPH_AMD_LIB=$PWD/ab/libcugraph_c_$v.so timeout -k 10 300 python -u scripts/mg_bfs_ab.py ${SCALE:-24} 40,64 > $OUT/$v$rep.txt 2>&1 || exit 1
    echo "$v$rep $(grep -E 'MG one' $OUT/$v$rep.txt)"
  done
done
