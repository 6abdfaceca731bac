set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02v5_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r02v5_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02v5_gpu_tests.log
bash tools/profile_round.sh gpurun_out/prof_r02v5 || exit 1
python3 tools/step_breakdown.py gpurun_out/prof_r02v5/bench > gpurun_out/prof_r02v5/step_breakdown.txt
timeout -k 10 300 python bench.py > gpurun_out/r02v5_bench_full.json 2> gpurun_out/r02v5_bench_full.err || exit 1
tail -1 gpurun_out/r02v5_bench_full.json | cut -c1-200
