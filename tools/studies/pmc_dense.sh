# The dense wave kernels (tools/studies/dense_bench.py, 16^4 12x12 complex<double>): SQ counters
# of every dispatch, one rocprofv3 pass per counter set; run on the GPU box from the repo root.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc_dense
mkdir -p $O
export CASES=site12 WAVE=2 PYTHONPATH=$R/tools/studies
n=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
         "SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
         "SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc$n -o run -- python3 $R/tools/studies/dense_bench.py > $O/pmc$n.log 2>&1
done
