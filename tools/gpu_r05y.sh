# host timeline of C4 with the checks' set-up phases marked
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05y
mkdir -p $O
cd $R
QVQ_HOST_TRACE=1 QVQ_CERT_TRACE=1 timeout -k 10 120 python3 tools/quick_timing.py 4096,4,12 > $O/c4_host.log 2>&1 || exit $?
python3 - <<'PY'
t=open('gpurun_out/r05y/c4_host.log').read().split('qvq host trace:')[-1].split('\n{')[0]
for l in t.strip().splitlines():
    if any(x in l for x in ('K2048','K4096','results','joined','return')): print(l)
PY
grep "qvq kahan: K 4096" $O/c4_host.log | tail -1
