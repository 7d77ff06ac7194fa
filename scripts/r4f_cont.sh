# Round 4 (f): the step tail's hot-run continuation as per-thread sums (one butterfly at the end,
# two chunks of loads per round): correctness (fused-kernel + DP tests), the default bench, the
# reference's k = 32 shapes, and the bench's secondary windows with the TFRecord window first (x2)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/b200_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $O/nb_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 > $O/rd_$r.log 2>&1
done
ROCFM_BENCH_TF_FIRST=1 timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/b20_tffirst_1.log 2>&1
ROCFM_BENCH_TF_FIRST=1 timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/b20_tffirst_2.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b200 -o b200 -- python3 bench.py --steps 200 --warmup 20 --no_secondary > $O/prof_b200.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nb -o nb -- python3 bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $O/prof_nb.log 2>&1
