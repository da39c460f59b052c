# 12x12 BSR (bsr_mfma_dma_kernel): SQ cycle breakdown, MFMA busy and clock, one counter pass
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r2c_c
cd /tmp && export TMPDIR=/tmp
MODES=1 ROUNDS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/r2c_c/pmc -o run -- python3 $R/tools/bsr_blk_sweep.py > $R/gpurun_out/r2c_c/pmc.log 2>&1
echo done
