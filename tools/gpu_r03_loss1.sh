# A/B: loss forward+backward in one call (finalize on the backward launch) vs two calls; loss tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3 4; do
  for v in split fused; do
    F=""; [ $v = split ] && F="--loss-split"
    timeout -k 10 240 python -u tools/variant_step.py --tag $v $F --steps 60 >> gpurun_out/r03_loss1.jsonl 2>> gpurun_out/r03_loss1.err || { tail -20 gpurun_out/r03_loss1.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_loss1.jsonl"):
    d = json.loads(l); print(d["tag"], d["ms_per_step"])
P
timeout -k 10 600 python -u -m pytest tests/test_loss_gpu.py tests/test_fused_gpu.py tests/test_sharded_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_loss1_tests.log 2>&1 || { tail -30 gpurun_out/r03_loss1_tests.log; exit 1; }
tail -1 gpurun_out/r03_loss1_tests.log
