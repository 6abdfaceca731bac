set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_parity_gpu.py::test_forced_large_frame_paths tests/test_fullsize_gpu.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r03_t1.log 2>&1 || { tail -60 gpurun_out/r03_t1.log; exit 1; }
grep -E "PASS|FAIL|rel L1|low_pass|passed|failed" gpurun_out/r03_t1.log | tail -30
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03_b1.json 2> gpurun_out/r03_b1.err || { tail -30 gpurun_out/r03_b1.err; exit 1; }
cat gpurun_out/r03_b1.json | cut -c1-1500
