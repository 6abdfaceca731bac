# A/B: duplicate window starts + range clearing inside the pair-count scan (marks) vs the
# window-starts launch (base); full -m gpu suite; the step's launch sequence
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3 4; do
  for v in base marks2; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 60 >> gpurun_out/r03_marks2.jsonl 2>> gpurun_out/r03_marks2.err || { tail -20 gpurun_out/r03_marks2.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_marks2.jsonl"):
    d = json.loads(l); s = d["stages_ms"]; print(d["tag"], d["ms_per_step"], s.get("scan"), s.get("duplicate"))
P
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_marks2_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r03_marks2_suite.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03_marks2_prof -o run --output-format csv -- python3 tools/variant_step.py --tag seq --steps 30 > gpurun_out/r03_marks2_step.json 2> gpurun_out/r03_marks2_prof.err || { tail -20 gpurun_out/r03_marks2_prof.err; exit 1; }
python3 tools/step_breakdown.py gpurun_out/r03_marks2_prof --first 33 --count 25 --seq > gpurun_out/r03_marks2_seq.txt 2>&1
head -20 gpurun_out/r03_marks2_seq.txt
