# C4 per-level host tree build times (quick_timing tree_ms) with the checks' helper threads at
# 8 (default), 1, and with no checks (QVQ_KAHAN=0): is the level-12 tree slowed by the checks?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05t
mkdir -p $O
cd $R
show() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2 wall', d['wall_ms'], 'tree', d['tree_ms'][-3:], 'other', d['other_ms'][-3:])"; }
timeout -k 10 120 python3 tools/quick_timing.py 4096,4,12 > $O/def.log 2>&1 && show $O/def.log default
QVQ_CERT_THREADS=1 timeout -k 10 120 python3 tools/quick_timing.py 4096,4,12 > $O/t1.log 2>&1 && show $O/t1.log threads1
QVQ_KAHAN=0 timeout -k 10 120 python3 tools/quick_timing.py 4096,4,12 > $O/ex.log 2>&1 && show $O/ex.log exactsum
timeout -k 10 120 python3 tools/quick_timing.py 4096,4,12 > $O/def2.log 2>&1 && show $O/def2.log default2
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
