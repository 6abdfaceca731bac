# tests + bench trace of the tree, then the gauss_bwd compact-row A/B (gpurun_variants gb_base / gb_compact)
set -o pipefail
TAG=$1
bash tools/gpu_r04q.sh $TAG || exit 1
bash tools/gpu_ab.sh $TAG "gb_base gb_compact"
