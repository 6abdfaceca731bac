mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for impl in 0 2; do
RAIN_FWD_IMPL=$impl timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_fwd_$impl -o run --output-format csv -- python3 tools/pmc_workload.py > gpurun_out/pmc_fwd_$impl.log 2>&1 || exit 1
done
