# Round 5 bench: the default bench line, then the C3-only bench under rocprofv3 (kernel stats).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05f
mkdir -p $O
cd $R
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o c3 -- python3 $R/bench.py --steps 20 --warmup 3 --c5-steps 0 --c4-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline > $O/c3_bench.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
echo done
