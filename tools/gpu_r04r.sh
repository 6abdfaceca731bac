# early-stop split A/B with the gather phase B
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for o in early_den=3 early_den=4 early_den=5 early_den=2; do
    timeout -k 10 300 python -u tools/variant_step.py --tag $o --tune $o \
      >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || { tail -20 gpurun_out/${TAG}_ab.err; exit 1; }
  done
done
cat gpurun_out/${TAG}_ab.jsonl
