# Round 4 (p): the driver-shaped bench with secondary windows and the default bench, after the
# DPP scan; kernel trace of the default bench
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/b20.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_ns.log 2>&1
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b200 -- python3 bench.py --steps 200 --warmup 20 --no_secondary > $O/prof.log 2>&1
