# Round 6 (l): TFRecord-fed window — five processes (rate, GPU-side stall), and one memory-copy trace
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6l
mkdir -p $O
R=$GRAFT_REPO_ROOT
TF="python bench.py --gpus 1 --input tfrecord --steps 2048 --warmup 128 --steps_per_graph 32"
for rep in 1 2 3 4 5; do
  timeout -k 10 200 $TF > $O/tf_$rep.json 2> $O/tf_$rep.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/p_tf -o run -- python3 $R/bench.py --gpus 1 --input tfrecord --steps 2048 --warmup 128 --steps_per_graph 32 > $R/$O/prof_tf.log 2>&1 || exit 1
python3 $R/tools/rocpd_copies.py $(find /tmp/p_tf -name "*.db" | head -1) > $R/$O/copies.txt 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $(find /tmp/p_tf -name "*.db" | head -1) > $R/$O/kernels.txt 2>&1 || exit 1
