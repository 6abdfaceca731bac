set -o pipefail
mkdir -p gpurun_out/p1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 60 rocprofv3 -L > gpurun_out/p1/counters.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/p1/stall -o run --output-format csv -- python3 tools/pmc_workload.py > gpurun_out/p1/stall.log 2>&1
python3 tools/pmc_stalls.py gpurun_out/p1/stall > gpurun_out/p1/stalls.txt 2>&1
head -40 gpurun_out/p1/stalls.txt
