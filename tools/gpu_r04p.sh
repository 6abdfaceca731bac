# round-4 profile passes of the current tree (kernel trace + stats of the default bench, PMC passes)
set -o pipefail
TAG=$1
bash tools/profile_round.sh gpurun_out/${TAG} || exit 1
python3 tools/step_breakdown.py gpurun_out/${TAG}/bench --window > gpurun_out/${TAG}/timed_kernels.txt 2>&1
python3 tools/step_breakdown.py gpurun_out/${TAG}/bench --window --seq | tail -40 > gpurun_out/${TAG}/launch_sequence.txt 2>&1
head -30 gpurun_out/${TAG}/timed_kernels.txt
cat gpurun_out/${TAG}/pmc_traffic.json | head -60
