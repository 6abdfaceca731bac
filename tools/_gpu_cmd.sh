set -o pipefail
mkdir -p gpurun_out
for v in head nog head nog; do
  if [ $v = head ]; then L=""; else L=$PWD/gpurun_variants/$v.so; fi
  RAIN_RASTER_LIB=$L timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > gpurun_out/b_$v.json 2> gpurun_out/b_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/b_$v.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$v',d['value'],d['ms_per_step'],k['duplicate']['ms_per_step'],k['tile_sort']['ms_per_step'])"
done
