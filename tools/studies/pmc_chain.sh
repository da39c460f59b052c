# The chain contraction's GEMM (tools/studies/chain_contraction.py, T48 forms): kernel trace + SQ counters
# (MFMA busy, wait cycles), each counter set in its own rocprofv3 pass; run on the GPU box from the
# repo root.  Summaries: tools/prof_summary.py on the .db, the csv files as they are.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc_chain
mkdir -p $O
export T48=${T48:-6}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/tools/studies/chain_contraction.py > $O/trace.log 2>&1
n=0
for c in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAVES" "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VMEM_RD SQ_WAIT_ANY"; do
  n=$((n + 1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/pmc$n -o run -- python3 $R/tools/studies/chain_contraction.py > $O/pmc$n.log 2>&1
done
