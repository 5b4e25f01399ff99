# C4 with the reference's rule: what the checks cost -- helper threads, synchronous levels, the
# exact-sum rule (no checks)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05u
mkdir -p $O
cd $R
B="--steps 5 --warmup 2 --c4-steps 8 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $B > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', 'C3', d['ms_per_step'], 'C4', d['c4']['ms_per_step'])"
}
run default QVQ_X=0 && run threads8 QVQ_CERT_THREADS=8 && run threads2 QVQ_CERT_THREADS=2 && run exactsum QVQ_KAHAN=0 && run default2 QVQ_X=0
QVQ_CERT_TRACE=1 timeout -k 10 120 python3 tools/quick_timing.py 4096,4,12 > $O/c4_cert.log 2>&1; grep "qvq kahan" $O/c4_cert.log | tail -8
