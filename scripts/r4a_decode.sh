# Round 4 (a): device-side Example parsing, TFRecord-fed bench windows, headline + secondaries,
# merge on uncached memory, k=32 shapes (dedup x wide wgrad tiles A/B)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -v --timeout 120 --timeout-method thread > $O/decode_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 --loader_threads 4 > $O/tf_t4.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 --loader_threads 8 > $O/tf_t8.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 --loader_threads 16 --host_decode > $O/tf_host16.log 2>&1
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/b20.log 2>&1
timeout -k 10 300 python tools/bench_merge.py --worlds 2,4,8 --memory cached,uncached --skip_owner --iters 100 > $O/merge_mem.log 2>&1
timeout -k 10 300 python tools/bench_merge.py --worlds 8 --memory cached,uncached --cap 39936 --skip_owner --iters 100 > $O/merge_cap.log 2>&1
for D in 0 1; do for L in 128,64,32 256,128,64; do for T in auto 1; do
if [ $T = auto ]; then unset ROCFM_WGRAD_TW; else export ROCFM_WGRAD_TW=$T; fi
ROCFM_DEDUP=$D timeout -k 10 200 python bench.py --steps 200 --warmup 20 --embedding_size 32 --deep_layers $L --feature_size 117581 --no_secondary > $O/k32_${L//,/-}_dedup${D}_tw$T.log 2>&1
done; done; done
