# full -m gpu suite, bin-run statistics, dup_tile_order A/B (in-tree library), bench kernel trace
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bin_stats.py > gpurun_out/${TAG}_bin_stats.json 2> gpurun_out/${TAG}_bin_stats.err \
  || { tail -20 gpurun_out/${TAG}_bin_stats.err; exit 1; }
for r in 1 2; do
  for o in dup_tile_order=1 dup_tile_order=0 sort_min_units_tile=2048 early_den=2 early_den=4; do
    timeout -k 10 300 python -u tools/variant_step.py --tag $o --tune $o \
      >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || { tail -20 gpurun_out/${TAG}_ab.err; exit 1; }
  done
done
cat gpurun_out/${TAG}_ab.jsonl
bash tools/gpu_r04f.sh $TAG
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_api -o run --output-format csv \
  -- python3 tools/api_trace.py > gpurun_out/${TAG}_api.log 2> gpurun_out/${TAG}_api.err || { tail -20 gpurun_out/${TAG}_api.err; exit 1; }
cat gpurun_out/${TAG}_api.log
python3 tools/step_breakdown.py gpurun_out/${TAG}_api --window > gpurun_out/${TAG}_api_kernels.txt 2>&1
python3 tools/step_breakdown.py gpurun_out/${TAG}_api --window --seq | tail -60 > gpurun_out/${TAG}_api_seq.txt 2>&1
head -30 gpurun_out/${TAG}_api_kernels.txt
