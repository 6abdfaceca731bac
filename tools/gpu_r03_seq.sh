# cov2D association change: parity + full GPU suite; kernel-trace of the training step, launch sequence
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_seq_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r03_seq_suite.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03_seq_prof -o run --output-format csv -- python3 tools/variant_step.py --tag seq --steps 30 > gpurun_out/r03_seq_step.json 2> gpurun_out/r03_seq_prof.err || { tail -20 gpurun_out/r03_seq_prof.err; exit 1; }
python3 tools/step_breakdown.py gpurun_out/r03_seq_prof --first 5 --count 50 --seq > gpurun_out/r03_seq.txt 2>&1
head -80 gpurun_out/r03_seq.txt
