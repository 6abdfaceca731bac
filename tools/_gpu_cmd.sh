set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_fused_gpu.py tests/test_early_stop_gpu.py tests/test_aux_normal_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
for v in head prev head prev; do
  if [ $v = head ]; then L=""; else L=$PWD/gpurun_variants/$v.so; fi
  RAIN_RASTER_LIB=$L timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline > gpurun_out/b_$v.json 2> gpurun_out/b_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/b_$v.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$v',d['value'],d['ms_per_step'],k['blend_fwd']['ms_per_step'],k['blend_bwd']['ms_per_step'])"
done
