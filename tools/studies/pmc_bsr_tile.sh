# Counters of the 3x3 9-point BSR kernels at 16^4, n = 64 (tools/studies/bsr_bound.py): the
# row-chunk kernel (bsr.tile 0) against the site-tile kernels (bsr.tile 1: 16 sites x 8 columns,
# 2: 8 sites x 16 columns) -- fabric bytes
# (FETCH_SIZE), the vector-memory path (TA busy, L1 -> L2 requests) and the LDS (instructions,
# bank conflicts, issue stalls).  One rocprofv3 pass per counter group; run on the GPU box from
# the repo root; per-dispatch tables by tools/studies/pmc_kernels.py.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc_tile
mkdir -p $O
export L=16 KINDS=stencil NCOLS=64 TILES=0,1,2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/tools/studies/bsr_bound.py > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_sum TCP_TCC_READ_REQ_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/sq -o run -- python3 $R/tools/studies/bsr_bound.py > $O/sq.log 2>&1
for p in fetch sq; do
  f=$(ls $O/$p/*/run_counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] || f=$(find $O/$p -name '*counter_collection.csv' | head -1)
  echo "== $p (row chunks: bsr_ell9_kernel)"; python3 $R/tools/studies/pmc_kernels.py "$f" bsr_ell9_kernel | tail -3
  echo "== $p (site tiles 16x8: bsr_ell9_tile_kernel<., 16, 8>)"; python3 $R/tools/studies/pmc_kernels.py "$f" ", 16, 8>" | tail -3
  echo "== $p (site tiles 8x16: bsr_ell9_tile_kernel<., 8, 16>)"; python3 $R/tools/studies/pmc_kernels.py "$f" ", 8, 16>" | tail -3
done > $O/summary.txt
