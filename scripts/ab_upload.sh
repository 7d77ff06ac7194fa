# A/B of hipGraphUpload after capture (ROCFM_GRAPH_UPLOAD) on the driver-shaped 20-step window.
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for u in 0 1; do
    ROCFM_GRAPH_UPLOAD=$u timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no_secondary > gpurun_out/r3_up${u}_b20_$i.log 2>&1
  done
done
ROCFM_GRAPH_UPLOAD=1 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no_secondary > gpurun_out/r3_up1_b200.log 2>&1
