# Aggregate TFRecord decode rate of 1/2/4/8 concurrent loader processes (one per rank shard) on the
# GPU box's host share, record vs file sharding, and the decoded on-disk cache (no GPU use).
set -e
cd $GRAFT_REPO_ROOT
nproc > gpurun_out/r3_la_nproc.txt
timeout -k 10 600 python -u tools/loader_aggregate.py --procs 1,2,4,8 --threads 2 --records 4000000 --files 16 \
  --json gpurun_out/r3_loader_aggregate_box.json > gpurun_out/r3_loader_aggregate_box.log 2>&1
