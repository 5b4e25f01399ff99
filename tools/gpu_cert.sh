# Kahan-rule parity (tie certificate + evaluator), per-level timings of C2/C3/C4, then the C3 trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
bash tools/gpu_kahan2.sh || exit 1
QVQ_KAHAN_DEBUG=1 timeout -k 10 200 python3 tools/quick_timing.py > gpurun_out/qt.log 2>&1 || { tail -20 gpurun_out/qt.log; exit 1; }
grep '^{' gpurun_out/qt.log | cut -c1-400
grep "qvq kahan" gpurun_out/qt.log | sort | uniq -c | head -20
bash tools/gpu_c3trace.sh
