# Kahan tests, then the C3 trace (tools/gpu_c3trace.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_kahan2.sh && bash tools/gpu_c3trace.sh
