# Kernel trace of C3 quantizes (quick_timing) with the per-level timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
QVQ_KAHAN_DEBUG=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c3t -o t -- python3 $R/tools/quick_timing.py ${1:-4096,2,10} > $R/gpurun_out/c3t.log 2>&1 || { tail -20 $R/gpurun_out/c3t.log; exit 1; }
cat $R/gpurun_out/c3t.log | grep '^{'
python3 $R/tools/trace_view.py $R/gpurun_out/c3t/t_kernel_trace.csv --compact 2>&1 | tail -60
grep "qvq kahan" $R/gpurun_out/c3t.log | sort | uniq -c | head
python3 - $R/gpurun_out/c3t/t_kernel_trace.csv <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name']
    if 'ks_' in n or 'rocclr' in n:
        key = n.split('(')[0].split('::')[-1][:40]
        d[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items(), key=lambda x: -sum(x[1])):
    print("%-42s n=%3d mean=%8.1f max=%8.1f us" % (k, len(v), sum(v) / len(v), max(v)))
PY
