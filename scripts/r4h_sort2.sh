# Round 4 (h): the scatter kernel computes its own digit offsets (no scan launch): sort tests,
# the TFRecord window and driver-shaped bench, kernel traces; phase stamps after the continuation
# change (default and reference-default shapes) and the widened wgrad tiles at the reference
# defaults again (the hot-run continuation no longer bounds the tail's embedding role)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sort_gpu.py tests/test_rowshard_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_$r.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 > $O/tf_s16_$r.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 128 --steps_per_graph 32 > $O/tf_s32_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 > $O/rd_$r.log 2>&1
ROCFM_WGRAD_TW=auto timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 > $O/rd_twauto_$r.log 2>&1
done
MULTI=1 timeout -k 10 300 python tools/diag_phases.py > $O/phases_default.log 2>&1
MULTI=1 K=32 V=117581 LAYERS=256,128,64 GENERIC=1 timeout -k 10 300 python tools/diag_phases.py > $O/phases_refdef.log 2>&1
MULTI=1 K=32 V=117581 LAYERS=128,64,32 GENERIC=1 timeout -k 10 300 python tools/diag_phases.py > $O/phases_nb.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tf -o tf -- python3 bench.py --input tfrecord --steps 2048 --warmup 64 > $O/prof_tf.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nb -o nb -- python3 bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $O/prof_nb.log 2>&1
