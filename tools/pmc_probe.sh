set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc/a -o a -- python3 $R/benchmarks/kernel_probe.py conv3_fwd conv2_dgrad conv1_fwd conv2_fwd > $R/gpurun_out/pmc/a.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM --kernel-trace --output-format csv -d $R/gpurun_out/pmc/b -o b -- python3 $R/benchmarks/kernel_probe.py conv3_fwd conv2_dgrad conv1_fwd conv2_fwd > $R/gpurun_out/pmc/b.log 2>&1
