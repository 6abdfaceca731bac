mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python tools/step_ab.py --knob fwd_impl --values 0,2 --blocks 4 --steps 40 --stages > gpurun_out/ab_fwd.txt 2>&1 || exit 1
timeout -k 10 300 python tools/step_ab.py --knob gauss_bwd_split --values 0,1 --blocks 4 --steps 40 --stages > gpurun_out/ab_split.txt 2>&1 || exit 1
RAIN_GAUSS_BWD_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_split -o run --output-format csv -- python3 tools/pmc_workload.py > gpurun_out/prof_split.log 2>&1 || exit 1
timeout -k 10 200 python tools/raster_ab.py --knob fwd_impl --values 2 --rounds 5 > gpurun_out/fold1.json 2>&1 || exit 1
RAIN_RASTER_LIB=$PWD/gpurun_variants/nofold.so timeout -k 10 200 python tools/raster_ab.py --knob fwd_impl --values 2 --rounds 5 > gpurun_out/fold0.json 2>&1
