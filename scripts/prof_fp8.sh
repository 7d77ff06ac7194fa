# rocprofv3 kernel traces of the bench step, bf16 vs fp8 compute (200 steps each).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_fp8
for dt in bf16 fp8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fp8 -o $dt -- python3 bench.py --steps 200 --warmup 20 --no_secondary --compute_dtype $dt > gpurun_out/prof_fp8/bench_$dt.log 2>&1
done
