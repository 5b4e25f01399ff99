# C4 (4x4 blocks, D=48) per-level traces at three VALU/MFMA crossover points (QVQ_WIDE_MIN_K).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/ab_env.sh 4096,4,12 "w32:QVQ_WIDE_MIN_K=32" "w64:QVQ_WIDE_MIN_K=64" "w128:QVQ_WIDE_MIN_K=128"
