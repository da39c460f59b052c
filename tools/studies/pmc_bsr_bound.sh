# Fabric bytes of the 3x3 BSR kernel per x-reuse case (tools/studies/bsr_bound.py): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 passes; run on the GPU box from the repo root; summarise with
# tools/pmc_summary.py.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc_bound
mkdir -p $O
export KINDS=${KINDS:-stencil,local,self} NCOLS=${NCOLS:-12,64}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/tools/studies/bsr_bound.py > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/tools/studies/bsr_bound.py > $O/write.log 2>&1
