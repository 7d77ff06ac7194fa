# Round 5 (n): kernel traces of the k = 32 shapes (notebook, flag defaults with the split), the
# TFRecord window order with the ring zero-fill race re-introduced (ROCFM_HAZARD_INJECT=ring_init)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_notebook -o nb -- python3 bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --no_secondary > $O/notebook_prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_refdef -o rd -- python3 bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 --no_secondary > $O/refdef_prof.log 2>&1 || exit 1
ROCFM_HAZARD_INJECT=ring_init ROCFM_BENCH_TF_TWICE=1 timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_tftwice_raceinject.log 2>&1 || exit 1
ROCFM_BENCH_TF_FIRST=0 timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_tflast.log 2>&1 || exit 1
