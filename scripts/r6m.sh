# Round 6 (m): full GPU suite, smoke, the driver-shaped bench with its secondary windows;
# fp8 vs bf16 row-kernel phases; notebook kernel trace
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6m
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.json 2> $O/b20.err || exit 1
MULTI=1 DTYPE=fp8 timeout -k 10 200 python tools/diag_phases.py > $O/phases_default_fp8.txt 2>&1 || exit 1
MULTI=1 DTYPE=bf16 timeout -k 10 200 python tools/diag_phases.py > $O/phases_default_bf16.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/p_nb -o run -- python3 $R/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $R/$O/prof_nb.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $(find /tmp/p_nb -name "*.db" | head -1) > $R/$O/prof_nb.txt 2>&1 || exit 1
