# Round 4 (c): onesweep vs merge-path radix sort on the side chain (A/B, interleaved), the
# driver-shaped bench with its secondary windows, correctness of the onesweep path, and the loader
# aggregate over a longer window (8 processes, record sharding through the index)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4c
mkdir -p $O
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/ab_auto_$r.log 2>&1
ROCFM_RADIX=onesweep timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/ab_onesweep_$r.log 2>&1
done
ROCFM_RADIX=onesweep timeout -k 10 300 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > $O/onesweep_tests.log 2>&1
ROCFM_RADIX=onesweep timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/onesweep_smoke.log 2>&1
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/b20.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ROCFM_RADIX=onesweep timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_os -o os -- python bench.py --steps 200 --warmup 20 --no_secondary > $O/prof_os.log 2>&1
timeout -k 10 600 python tools/loader_aggregate.py --procs 1,8 --threads 2 --records 6400000 --modes raw --shard_policy record --json $O/loader_agg.json > $O/loader_agg.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 --loader_threads 4 > $O/tf_t4.log 2>&1
ROCFM_RADIX=onesweep timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 --loader_threads 4 > $O/tf_t4_onesweep.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tf -o tf -- python bench.py --input tfrecord --steps 2048 --warmup 64 --loader_threads 4 > $O/prof_tf.log 2>&1
