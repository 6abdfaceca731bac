# SSIM band-height A/B: kernel times (tools/loss_ab.py), then the loss parity tests per variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in lb32 lbb64 lbb48 lbf48 lbb32la6 lbf32la3; do
    timeout -k 10 120 python -u tools/loss_ab.py --lib gpurun_variants/$v.so >> gpurun_out/r03_ssim_ab2.jsonl 2>> gpurun_out/r03_ssim_ab2.err || { tail -20 gpurun_out/r03_ssim_ab2.err; exit 1; }
  done
done
cat gpurun_out/r03_ssim_ab2.jsonl
for v in lbb64 lbf48; do
  RAIN_LOSS_LIB=gpurun_variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_loss_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_ssim_${v}.log 2>&1 || { tail -20 gpurun_out/r03_ssim_${v}.log; exit 1; }
  tail -1 gpurun_out/r03_ssim_${v}.log
done
