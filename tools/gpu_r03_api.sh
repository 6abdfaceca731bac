set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/variant_step.py --tag base --api > gpurun_out/r03_api.json 2> gpurun_out/r03_api.err || { tail -20 gpurun_out/r03_api.err; exit 1; }
cat gpurun_out/r03_api.json
