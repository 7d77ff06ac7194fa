# PMC counters of the default bench's kernels (two passes, counters only with --kernel-trace)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c/pmc
echo start > gpurun_out/r3c/pmc/status.txt
timeout -k 10 200 python -c "import torch; torch.zeros(1, device='cuda')" > /dev/null 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "deepfm_rows|step_tail" --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r3c/pmc/p1 -o p1 -- python3 bench.py --steps 20 --warmup 5 --no_secondary > gpurun_out/r3c/pmc/p1.log 2>&1
echo p1 done >> gpurun_out/r3c/pmc/status.txt
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "deepfm_rows|step_tail" --pmc FETCH_SIZE TCC_HIT_sum SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/r3c/pmc/p2 -o p2 -- python3 bench.py --steps 20 --warmup 5 --no_secondary > gpurun_out/r3c/pmc/p2.log 2>&1
echo p2 done >> gpurun_out/r3c/pmc/status.txt
