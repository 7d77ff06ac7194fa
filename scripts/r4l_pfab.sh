# Round 4 (l): the tail's prefetch through one code path: per-step ≡ graphs (bitwise), prefetch
# on / off in the same process, GPU suites, bench A/B
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4l
mkdir -p $O
STEPS=40 timeout -k 10 200 python tools/diag_determinism.py > $O/det40.log 2>&1
PREFETCH_AB=1 STEPS=40 timeout -k 10 200 python tools/diag_determinism.py > $O/ab40.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_bf16_table_gpu.py tests/test_sort_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/b200_pf_$r.log 2>&1
ROCFM_TAIL_PREFETCH=0 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/b200_nopf_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_pf_$r.log 2>&1
ROCFM_TAIL_PREFETCH=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_nopf_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $O/nb_pf_$r.log 2>&1
ROCFM_TAIL_PREFETCH=0 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $O/nb_nopf_$r.log 2>&1
done
MULTI=1 timeout -k 10 300 python tools/diag_phases.py > $O/phases_default.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_fused_dp_gpu.py tests/test_rowshard_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_dist.log 2>&1
