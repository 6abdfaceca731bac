mkdir -p gpurun_out
timeout -k 10 120 python tools/phaseb_stats.py > gpurun_out/phaseb_stats.json 2>&1 || exit 1
timeout -k 10 120 python tools/fwd_check.py --impls 0,2 --points 100000 --width 800 --height 800 > gpurun_out/fwd_check.txt 2>&1 || exit 1
timeout -k 10 200 python tools/raster_ab.py --knob fwd_impl --values 0,2 --rounds 5 > gpurun_out/skip1.json 2>&1 || exit 1
for v in noskip skipg8; do
RAIN_RASTER_LIB=$PWD/gpurun_variants/$v.so timeout -k 10 200 python tools/raster_ab.py --knob fwd_impl --values 2 --rounds 5 > gpurun_out/$v.json 2>&1 || exit 1
done
