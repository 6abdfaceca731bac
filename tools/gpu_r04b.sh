# Round-4 GPU call: launch-cost probe (+ its rocprofv3 kernel trace), the -m gpu suite on the default
# build, then an interleaved A/B of two librain_raster.so variants (tools/variant_step.py).
#   bash tools/gpu_r04b.sh TAG VARIANT_A VARIANT_B [suite]
set -o pipefail
TAG=$1; VA=$2; VB=$3; SUITE=$4
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -x tools/launch_probe ] && [ ! -s gpurun_out/${TAG}_launch_probe.jsonl ]; then
  timeout -k 10 120 ./tools/launch_probe > gpurun_out/${TAG}_launch_probe.jsonl || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_lp -o lp --output-format csv \
    -- ./tools/launch_probe > /dev/null || exit 1
fi
if [ "$SUITE" = suite ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_gpu_tests.log
fi
for v in $VA $VB $VA $VB; do
  RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 300 python -u tools/variant_step.py --tag $v \
    >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || { tail -20 gpurun_out/${TAG}_ab.err; exit 1; }
done
cat gpurun_out/${TAG}_ab.jsonl
