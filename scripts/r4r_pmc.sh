# Round 4 (r): counters of the row kernel and the step tail after the DPP scan (one pass, 8 SQ)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "deepfm_rows|step_tail" --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O/p1 -o p1 -- python3 bench.py --steps 20 --warmup 5 --no_secondary > $O/p1.log 2>&1
