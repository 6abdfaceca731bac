set -o pipefail
mkdir -p gpurun_out
bash tools/profile_round.sh gpurun_out/prof_r02v3 || exit 1
python3 tools/step_breakdown.py gpurun_out/prof_r02v3/bench > gpurun_out/prof_r02v3/step_breakdown.txt
head -30 gpurun_out/prof_r02v3/step_breakdown.txt
