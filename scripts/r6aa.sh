# Round 6 (aa): full GPU suite, smoke, the driver-shaped bench with its secondary windows; kernel
# traces of the headline and notebook windows
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6aa
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.json 2> $O/b20.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/p_d -o run -- python3 $R/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary > $R/$O/prof_d.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $(find /tmp/p_d -name "*.db" | head -1) > $R/$O/prof_d.txt 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/p_nb -o run -- python3 $R/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $R/$O/prof_nb.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $(find /tmp/p_nb -name "*.db" | head -1) > $R/$O/prof_nb.txt 2>&1 || exit 1
