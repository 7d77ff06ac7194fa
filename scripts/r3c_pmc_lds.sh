# LDS bank conflicts of the row kernel by ablation (diag kernel: ABLATE 1 = no h0T store, 2 = no FM, 4 = no prefetch)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c/pmcl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for a in 0 1 2 4; do
  ABLATE=$a MULTI=1 timeout -s KILL 180 rocprofv3 --kernel-trace --kernel-include-regex "deepfm_rows" --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r3c/pmcl/a$a -o a$a -- python3 tools/diag_phases.py > gpurun_out/r3c/pmcl/a$a.log 2>&1
  echo "ablate $a done" >> gpurun_out/r3c/pmcl/status.txt
done
