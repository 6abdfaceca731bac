# A/B: phase-B open-tile bitmask from the phase-A blend (bits: no SAT launch, row-word rect test),
# bitsq = bits + the mailbox wait queries the stream only after 20 ms; then the full -m gpu suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in base bits bitsq dupb; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 60 >> gpurun_out/r03_bits.jsonl 2>> gpurun_out/r03_bits.err || { tail -20 gpurun_out/r03_bits.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_bits.jsonl"):
    d = json.loads(l); s = d["stages_ms"]; print(d["tag"], d["ms_per_step"], s.get("duplicate"), s.get("tile_sort"), s.get("ranges"), s.get("blend_fwd"))
P
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_bits_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r03_bits_suite.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03_bits_prof -o run --output-format csv -- python3 tools/variant_step.py --tag seq --steps 30 > gpurun_out/r03_bits_step.json 2> gpurun_out/r03_bits_prof.err || { tail -20 gpurun_out/r03_bits_prof.err; exit 1; }
python3 tools/step_breakdown.py gpurun_out/r03_bits_prof --first 33 --count 25 --seq > gpurun_out/r03_bits_seq.txt 2>&1
head -40 gpurun_out/r03_bits_seq.txt
