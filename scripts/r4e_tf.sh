# Round 4 (e): the TFRecord-fed window at 16 / 32 / 64 steps per graph (32 and 64 put the side
# chain's composite-key sort over rocPRIM's 1M-item limit onto its onesweep path, the path the
# pool-fed headline's 64-step graphs use), the bench's in-process TFRecord window before / after the
# other secondary windows, and a kernel trace (csv).  Larger-S runs last: set -e ends the script at
# the first failure with the earlier results kept.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 > $O/tf_s16_1.log 2>&1
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/b20.log 2>&1
ROCFM_BENCH_TF_FIRST=1 timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/b20_tffirst.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 --steps_per_graph 32 > $O/tf_s32_1.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 128 --steps_per_graph 64 > $O/tf_s64_1.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 > $O/tf_s16_2.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 64 --steps_per_graph 32 > $O/tf_s32_2.log 2>&1
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 128 --steps_per_graph 64 > $O/tf_s64_2.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tf32 -o tf32 -- python3 bench.py --input tfrecord --steps 2048 --warmup 64 --steps_per_graph 32 > $O/prof_tf32.log 2>&1
