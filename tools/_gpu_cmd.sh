mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_early_stop_gpu.py tests/test_fused_gpu.py tests/test_aux_normal_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/bins_tests.log 2>&1
rc=$?; [ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline > gpurun_out/bench_bins.json 2> gpurun_out/bench_bins.err || exit 1
RAIN_RASTER_LIB=$PWD/gpurun_variants/head.so timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err
