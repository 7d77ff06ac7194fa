# Round 6 (ab): wgrad weights / slots loaded before the MFMA loop (wpf) vs after the reduce (base)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ab
mkdir -p $O
SO=deepfm-tensorflow-distributed-training-on-amazon-sagemaker_amd/_rocfm_hip.cpython-310-x86_64-linux-gnu.so
cp ab/wpf.so $SO
timeout -k 10 400 python -u -m pytest tests/test_emb_plan_gpu.py tests/test_fused_kernels_gpu.py tests/test_trajectory_gpu.py tests/test_bf16_table_gpu.py tests/test_fused_dp_gpu.py -x -q --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || exit 1
NB="--embedding_size 32 --feature_size 117581"
B="python bench.py --gpus 1 --no_secondary"
for rep in 1 2 3; do
  for v in wpf base; do
    cp ab/$v.so $SO
    timeout -k 10 150 $B --steps 20 --warmup 5 > $O/${v}_d20_$rep.json 2>/dev/null || exit 1
    timeout -k 10 150 $B --steps 20 --warmup 5 $NB > $O/${v}_n20_$rep.json 2>/dev/null || exit 1
  done
done
for v in wpf base; do
  cp ab/$v.so $SO
  timeout -k 10 150 $B --steps 200 --warmup 20 > $O/${v}_d200.json 2>/dev/null || exit 1
  timeout -k 10 150 $B --steps 200 --warmup 20 $NB > $O/${v}_n200.json 2>/dev/null || exit 1
  MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_d_${v}.txt 2>&1 || exit 1
  K=32 V=117581 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_n_${v}.txt 2>&1 || exit 1
done
cp ab/wpf.so $SO
