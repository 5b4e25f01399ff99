"""Per-kernel durations of the Kahan path (k_kahan.hip + the hipCUB sort) in a rocprofv3 trace."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name']
    if 'kc_' in n or 'rocprim' in n:
        key = n.replace('qvq::(anonymous namespace)::', '').split('(')[0][:60]
        agg[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
tot = 0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print(f"n={len(v):3d} avg={sum(v) / len(v):10.1f}us max={max(v):10.1f}  {k}")
print(f"total {tot:.1f} us")
