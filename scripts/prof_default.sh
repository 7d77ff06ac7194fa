# rocprofv3 kernel trace of the default bench (200 steps) + in-kernel phase stamps (multi-step path)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3 -o default -- python3 bench.py --steps 200 --warmup 20 --no_secondary > gpurun_out/prof_r3/bench.log 2>&1
MULTI=1 timeout -k 10 300 python tools/diag_phases.py > gpurun_out/prof_r3/phases.log 2>&1
