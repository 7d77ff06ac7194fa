# Round 5 (c): wide-vocabulary debug + the swizzled-layout phase stamps and bench
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 300 python tools/debug_wide.py > $O/w100m_16.log 2>&1 || exit 1
S=64 timeout -k 10 300 python tools/debug_wide.py > $O/w100m_64.log 2>&1 || exit 1
K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef.txt 2>&1 || exit 1
ROCFM_WGRAD_TW=auto K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef_twauto.txt 2>&1 || exit 1
MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_default.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1
for k in 0 1 2 3 4 5 6 7; do timeout -k 10 120 python tools/probe_stream_queues.py $k pool >> $O/queues_pool.jsonl 2>/dev/null || exit 1; done
for k in 0 1 2 3; do timeout -k 10 180 python tools/probe_stream_queues.py $k tf >> $O/queues_tf.jsonl 2>/dev/null || exit 1; done
ABLATE=8 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_default_gridbarrier.txt 2>&1 || exit 1
