# Round 5 (d): coalesced wgrad-epilogue refresh (oracle tests), the 1B-row streamed-vs-per-step
# debug, phase stamps (tw 1 / auto), the in-launch grid-barrier price, TFRecord window order A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_trajectory_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
V=1000000000 S=64 MODES=raw,step timeout -k 10 400 python tools/debug_wide.py > $O/w1b_64.log 2>&1 || exit 1
K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef.txt 2>&1 || exit 1
ROCFM_WGRAD_TW=auto K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef_twauto.txt 2>&1 || exit 1
ROCFM_WGRAD_TW=auto K=32 V=117581 LAYERS=128,64,32 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_notebook_twauto.txt 2>&1 || exit 1
MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_default.txt 2>&1 || exit 1
ABLATE=8 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_default_gridbarrier.txt 2>&1 || exit 1
for tw in 1 auto; do ROCFM_WGRAD_TW=$tw timeout -k 10 300 python bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 --no_secondary > $O/refdef_tw$tw.log 2>&1 || exit 1; done
for tw in 1 auto; do ROCFM_WGRAD_TW=$tw timeout -k 10 300 python bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --no_secondary > $O/notebook_tw$tw.log 2>&1 || exit 1; done
ROCFM_BENCH_TF_FIRST=0 timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_tflast.log 2>&1 || exit 1
ROCFM_BENCH_TF_FIRST=1 timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_tffirst.log 2>&1 || exit 1
