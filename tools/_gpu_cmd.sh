set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/step_ab.py --knob bwd_waves --values 0,3,2 --blocks 4 --steps 40 --stages > gpurun_out/ab_bw.txt 2>&1 || { tail -20 gpurun_out/ab_bw.txt; exit 1; }
grep -v Warn gpurun_out/ab_bw.txt | tail -6
