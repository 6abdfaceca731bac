set -o pipefail
mkdir -p gpurun_out/hosttrace
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/hosttrace -o run --output-format csv -- python3 tools/variant_step.py --tag ht --steps 20 > gpurun_out/hosttrace/out.log 2>&1
ls -la gpurun_out/hosttrace/*
