#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc16a -o a -- python bench.py --steps 32 --warmup 16 > gpurun_out/p16a.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc16b -o b -- python bench.py --steps 32 --warmup 16 > gpurun_out/p16b.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc16c -o c -- python bench.py --steps 32 --warmup 16 > gpurun_out/p16c.log 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/pmc16a/a_counter_collection.csv gpurun_out/pmc16b/b_counter_collection.csv gpurun_out/pmc16c/c_counter_collection.csv > gpurun_out/pmc16_summary.txt; rm -f gpurun_out/pmc16*/*_counter_collection.csv; cat gpurun_out/pmc16_summary.txt
