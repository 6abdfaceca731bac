mkdir -p gpurun_out
timeout -k 10 120 python tools/fwd_check.py --impls 0,2 --points 100000 --width 800 --height 800 > gpurun_out/fwd_check.txt 2>&1 || exit 1
timeout -k 10 200 python tools/raster_ab.py --knob fwd_s_waves --values 2,1,4 --rounds 5 > gpurun_out/g4.json 2>&1 || exit 1
for g in 2 8; do
RAIN_RASTER_LIB=$PWD/gpurun_variants/g$g.so timeout -k 10 200 python tools/raster_ab.py --knob fwd_s_waves --values 2,1,4 --rounds 5 > gpurun_out/g$g.json 2>&1 || exit 1
done
timeout -k 10 300 python tools/step_ab.py --split 3,4,6,8 --blocks 4 --steps 50 > gpurun_out/split_ab.txt 2>&1
