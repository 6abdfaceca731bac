# the Gaussian-sharded step forced at world 1 over RCCL, with the CPU baseline on the line
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --force-dist > gpurun_out/${TAG}_bench_forced_dist.json 2> gpurun_out/${TAG}_bench_forced_dist.err \
  || { tail -20 gpurun_out/${TAG}_bench_forced_dist.err; exit 1; }
grep -o '"cpu_baseline": {[^}]*}' gpurun_out/${TAG}_bench_forced_dist.json
grep -o '"value": [0-9.]*' gpurun_out/${TAG}_bench_forced_dist.json | head -1
