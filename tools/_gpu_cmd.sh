set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_early_stop_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 300 python tools/step_ab.py --knob sort_min_units_tile --values 1024,512,2048 --blocks 4 --steps 40 --stages > gpurun_out/ab_units.txt 2>&1 || { tail -20 gpurun_out/ab_units.txt; exit 1; }
grep -v Warn gpurun_out/ab_units.txt | tail -6
