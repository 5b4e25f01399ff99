# Round 5 final record on the final tree (pruning from K = 256): bench.py default flags, the kernel
# stats of the same command and the PMC HBM passes (tools/gpu_bench.sh); the suite ran on this code
# in profiles/r05am
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && bash tools/gpu_bench.sh r05an || exit $?
echo record done
