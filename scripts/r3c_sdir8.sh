# search+dir at W = 4 / 8 with larger directories
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c/sdir8
for nb in 8192 16384 32768 65536; do
  timeout -k 10 200 python tools/bench_merge.py --worlds 4,8 --sdir_buckets $nb > gpurun_out/r3c/sdir8/nb$nb.log 2>&1
done
