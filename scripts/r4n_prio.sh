# Round 4 (n): the training stream at high priority over the side / copy streams (A/B, interleaved)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4n
mkdir -p $O
python -c "import torch; print(torch.cuda.Stream.priority_range())" > $O/range.log 2>&1
for r in 1 2; do
timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 128 --steps_per_graph 32 > $O/tf_base_$r.log 2>&1
ROCFM_MAIN_PRIORITY=1 timeout -k 10 300 python bench.py --input tfrecord --steps 2048 --warmup 128 --steps_per_graph 32 > $O/tf_prio_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_base_$r.log 2>&1
ROCFM_MAIN_PRIORITY=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_prio_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/b200_base_$r.log 2>&1
ROCFM_MAIN_PRIORITY=1 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/b200_prio_$r.log 2>&1
done
