set -o pipefail
mkdir -p gpurun_out
for v in base pref; do
  RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 300 python -u tools/owner_bench.py >> gpurun_out/r03_owner.jsonl 2>> gpurun_out/r03_owner.err || { tail -20 gpurun_out/r03_owner.err; exit 1; }
done
cat gpurun_out/r03_owner.jsonl
