set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS --kernel-trace -d gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 benchmarks/kernel_probe.py conv2_fwd conv3_fwd conv2_dgrad > gpurun_out/pmc/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 benchmarks/kernel_probe.py conv2_fwd conv3_fwd conv2_dgrad > gpurun_out/pmc/p2.log 2>&1
