# The -m gpu suite on the default build, then (unless the suite crashed: abort, segfault, time limit)
# another GPU step given as the remaining arguments.  Test failures (exit 1) do not stop the
# second step; crashes do.
#   bash tools/gpu_suite_then.sh TAG [TESTS] -- CMD...
set -o pipefail
TAG=$1; shift
TESTS=tests
if [ "$1" != "--" ]; then TESTS=$1; shift; fi
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -25 gpurun_out/${TAG}_gpu_tests.log | grep -E "PASS|FAIL|Error|error|passed|failed" | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite ended with $rc: stopping"; exit $rc; fi
if [ $# -gt 0 ]; then "$@" || exit $?; fi
exit $rc
