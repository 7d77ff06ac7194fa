# Round 4 (g): rocfm's segmented radix sort (seg_sort.hip) in place of rocPRIM on every
# (key, index) sort: correctness (sort tests vs torch.sort / rocPRIM, fused-kernel, row-shard
# route, Estimator streaming), the bench with each sort library (A/B), the TFRecord-fed window at
# 16 / 32 steps per graph, and a kernel trace of the driver-shaped run
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sort_gpu.py -x -v --timeout 120 --timeout-method thread > $O/sort_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_rowshard_gpu.py tests/test_estimator_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/b200_rocfm_$r.log 2>&1
ROCFM_SORT_LIB=rocprim timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/b200_rocprim_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_rocfm_$r.log 2>&1
ROCFM_SORT_LIB=rocprim timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_rocprim_$r.log 2>&1
done
for r in 1 2; do
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 > $O/tf_s16_$r.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 128 --steps_per_graph 32 > $O/tf_s32_$r.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b20 -o b20 -- python3 bench.py --steps 20 --warmup 5 --no_secondary > $O/prof_b20.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tf -o tf -- python3 bench.py --input tfrecord --steps 2048 --warmup 64 > $O/prof_tf.log 2>&1
