# repeated quantizes on one context (tools/repeat_diag.py) under the default schedule, with the
# per-level timing events, and with the certificate preparation off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05j
mkdir -p $O
cd $R
timeout -k 10 120 python3 tools/repeat_diag.py -2 > $O/rep_default.log 2>&1; echo "rc $?"; cat $O/rep_default.log | grep -v Warn
timeout -k 10 120 python3 tools/repeat_diag.py -1 > $O/rep_timing.log 2>&1; echo "rc $?"; cat $O/rep_timing.log | grep -v Warn
QVQ_CERT_PREP=0 timeout -k 10 120 python3 tools/repeat_diag.py -2 > $O/rep_noprep.log 2>&1; echo "rc $?"; cat $O/rep_noprep.log | grep -v Warn
