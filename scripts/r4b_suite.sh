# Round 4 (b): the full GPU suite, the loader aggregate over 1..8 processes (record sharding through
# the record index; raw payloads vs host parse), and a kernel trace of the TFRecord-fed window
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
timeout -k 10 400 python tools/loader_aggregate.py --procs 1,2,4,8 --threads 2 --records 800000 --modes raw,tfrecord --shard_policy record --json $O/loader_agg.json > $O/loader_agg.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tf -o tf -- python bench.py --input tfrecord --steps 2048 --warmup 64 --loader_threads 4 > $O/prof_tf.log 2>&1
