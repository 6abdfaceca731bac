# full -m gpu suite + smoke of the current tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r03_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { tail -20 gpurun_out/r03_smoke.log; exit 1; }
tail -3 gpurun_out/r03_smoke.log
