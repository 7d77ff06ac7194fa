# Round 5 (pmc): counters of the flag-default row kernel, split vs unsplit (one pass each, 8 SQ + 1 GRBM)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NB="--steps 20 --warmup 5 --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 --no_secondary"
C="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "deepfm_rows" --pmc $C --output-format csv -d $O/split -o split -- python3 bench.py $NB > $O/split.log 2>&1 || exit 1
ROCFM_ROW_SPLIT=1 timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "deepfm_rows" --pmc $C --output-format csv -d $O/nosplit -o nosplit -- python3 bench.py $NB > $O/nosplit.log 2>&1 || exit 1
