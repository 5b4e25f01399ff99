# A/B of experimental libqvq builds: parity on the big fingerprints + per-level timings.
# usage: bash tools/ab.sh DIR1 DIR2 ...   (quant_amd/<DIR>/libqvq.so; "lib" = default build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ab
for d in "$@"; do
  export QVQ_LIB=$R/quant_amd/$d/libqvq.so
  echo "== $d"
  timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_scale.py $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fingerprint or s512 or beans or kodim or ties" > $R/gpurun_out/ab/pytest_$d.log 2>&1 || { tail -30 $R/gpurun_out/ab/pytest_$d.log; exit 1; }
  tail -1 $R/gpurun_out/ab/pytest_$d.log
  timeout -k 10 120 python $R/tools/quick_timing.py 4096,2,10 4096,4,12 > $R/gpurun_out/ab/quick_$d.log 2>&1 || exit 1
  python - $R/gpurun_out/ab/quick_$d.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    r=json.loads(l); print(r["S"],r["bw"],"total %.3f"%r["total_ms"],"assign",r["assign_ms"],"other",r["other_ms"],"upd",r["update_ms"])
PY
done
