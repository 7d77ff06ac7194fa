# rocprofv3 kernel traces of the bench with and without the per-tile dedup (tail chunk 256)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_dd
for dd in 0 1; do
  ROCFM_DEDUP=$dd ROCFM_TAIL_CHUNK=256 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dd -o dd$dd -- python3 bench.py --steps 200 --warmup 20 --no_secondary > gpurun_out/prof_dd/dd$dd.log 2>&1
done
