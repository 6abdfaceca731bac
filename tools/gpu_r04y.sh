# bounds from the bin sort vs a bounds launch: interleaved A/B
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for o in bounds_in_sort=1 bounds_in_sort=0; do
    timeout -k 10 300 python -u tools/variant_step.py --tag $o --tune $o \
      >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || { tail -20 gpurun_out/${TAG}_ab.err; exit 1; }
  done
done
cat gpurun_out/${TAG}_ab.jsonl
