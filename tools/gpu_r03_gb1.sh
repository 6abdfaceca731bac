# k_gauss_bwd A/B: param re-read bound (nopread, timing only), 64-thread workgroups, Adam batch 16
set -o pipefail
mkdir -p gpurun_out
for v in base nopread t64 b16 base; do
  RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 60 >> gpurun_out/r03_gb1.jsonl 2>> gpurun_out/r03_gb1.err || { tail -20 gpurun_out/r03_gb1.err; exit 1; }
done
cat gpurun_out/r03_gb1.jsonl
