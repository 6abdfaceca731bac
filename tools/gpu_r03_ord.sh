# A/B: backward tile order computed by an extra workgroup of the phase-B duplicate (ord) vs in the prologue (base); suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in base ord; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 60 >> gpurun_out/r03_ord3.jsonl 2>> gpurun_out/r03_ord3.err || { tail -20 gpurun_out/r03_ord3.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_ord3.jsonl"):
    d = json.loads(l); s = d["stages_ms"]; print(d["tag"], d["ms_per_step"], s.get("memset"), s.get("blend_bwd"))
P
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_ord3_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r03_ord3_suite.log; [ $rc -eq 0 ] || exit $rc
