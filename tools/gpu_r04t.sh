# cfg5 stress line (5M Gaussians, 4K, depth + normal) and the Gaussian-sharded step forced at world 1
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --points 5000000 --width 3840 --height 2160 --aux-normal --steps 30 --warmup 5 \
  --no-cpu-baseline > gpurun_out/${TAG}_cfg5_bench.json 2> gpurun_out/${TAG}_cfg5_bench.err \
  || { tail -20 gpurun_out/${TAG}_cfg5_bench.err; exit 1; }
cat gpurun_out/${TAG}_cfg5_bench.json
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 1 --force-dist --steps 50 --warmup 10 --no-cpu-baseline \
  > gpurun_out/${TAG}_forced_dist.json 2> gpurun_out/${TAG}_forced_dist.err || { tail -20 gpurun_out/${TAG}_forced_dist.err; exit 1; }
cat gpurun_out/${TAG}_forced_dist.json
