# A/B of librain_raster.so variants (tools/build_variant.py) on one box: two interleaved rounds of
# tools/variant_step.py per variant, then (with "pmc") one rocprofv3 SQ stall pass per variant over
# tools/pmc_workload.py, summarised by tools/pmc_stalls.py.
#   bash tools/gpu_ab.sh TAG "VARIANT ..." [pmc] [MATCH]
set -o pipefail
TAG=$1; VS=$2; PMC=$3; MATCH=${4:-blend_bwd}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in $VS; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 300 python -u tools/variant_step.py --tag $v \
      >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || { tail -20 gpurun_out/${TAG}_ab.err; exit 1; }
  done
done
cat gpurun_out/${TAG}_ab.jsonl
if [ "$PMC" = pmc ]; then
  for v in $VS; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU \
      GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/${TAG}_pmc_$v -o run --output-format csv \
      -- python3 tools/pmc_workload.py > /dev/null 2>> gpurun_out/${TAG}_pmc.err || { tail -20 gpurun_out/${TAG}_pmc.err; exit 1; }
    echo "== $v"; python3 tools/pmc_stalls.py gpurun_out/${TAG}_pmc_$v --match $MATCH
  done
fi
