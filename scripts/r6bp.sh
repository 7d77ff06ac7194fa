# Round 6 (bp): kernel traces of the final tree (headline and notebook, 200-step windows)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bp
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/p_d -o run -- python3 $R/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary > $R/$O/prof_d.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $(find /tmp/p_d -name "*.db" | head -1) > $R/$O/prof_d.txt 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/p_nb -o run -- python3 $R/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $R/$O/prof_nb.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $(find /tmp/p_nb -name "*.db" | head -1) > $R/$O/prof_nb.txt 2>&1 || exit 1
