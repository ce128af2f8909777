# The round call (pytest -m gpu, bench line, rocprof kernel stats) followed by BFS-only A/B runs
set -o pipefail
TAG=${TAG:-round} bash scripts/gpu_round.sh || exit $?
TAG=${TAG:-round}_ab MODES="${MODES:-- CGX_BFS_CONV_SYNC=1 - CGX_BFS_CONV_SYNC=1}" bash scripts/gpu_bfs_ab.sh
