# A/B of the mean kernel's grid cap (QVQ_MEAN_GRID) on C3: kernel traces + average duration.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/ab_env.sh 4096,2,10 "g128:QVQ_MEAN_GRID=128" "g256:QVQ_MEAN_GRID=256" "g512:QVQ_MEAN_GRID=512" > $R/gpurun_out/meanab.log 2>&1 || exit 1
python3 - $R <<'PY'
import csv, sys
for g in ["g128", "g256", "g512"]:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
         for r in csv.DictReader(open(sys.argv[1] + "/gpurun_out/abe/%s/t_kernel_trace.csv" % g)) if "mean_sums" in r["Kernel_Name"]]
    print(g, "mean_sums us:", [round(x, 1) for x in d])
PY
