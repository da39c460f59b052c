# The Kronecker BSR kernel (tools/studies/kron_bound.py, stencil, n = 12): kernel trace + SQ / TA / TD
# counters, each set in its own rocprofv3 pass; run on the GPU box from the repo root.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc_kron
mkdir -p $O
export KINDS=${KINDS:-stencil} NCOLS=${NCOLS:-12}
export PYTHONPATH=$R/tools
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/tools/studies/kron_bound.py > $O/trace.log 2>&1
n=0
for c in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" \
         "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD" \
         "TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64"; do
  n=$((n + 1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/pmc$n -o run -- python3 $R/tools/studies/kron_bound.py > $O/pmc$n.log 2>&1
done
