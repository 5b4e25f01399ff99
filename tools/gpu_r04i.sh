# final check of the tree as committed: smoke() and the GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r04i
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04i/smoke.log 2>&1 || { tail -5 gpurun_out/r04i/smoke.log; exit 1; }
tail -1 gpurun_out/r04i/smoke.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r04i/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04i/gpu_tests.log
exit $rc
