# C4 A/B: certificate replay threads
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r04h
nproc
for t in 8 4 16 2; do
QVQ_CERT_THREADS=$t timeout -k 10 120 python3 tools/c4_trace.py > gpurun_out/r04h/c4_t$t.log 2>&1 || exit 1
echo "threads=$t: $(grep -h 'quantize' gpurun_out/r04h/c4_t$t.log | tr '\n' ' ')"
done
