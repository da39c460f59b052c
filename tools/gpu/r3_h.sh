# round 3: PMC passes of the n = 64 3x3 BSR, row-chunk kernel vs one-wave-per-row kernel
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r3_h
cd /tmp && export TMPDIR=/tmp
export NS=64 FORMS=row_chunk,wave_pd2 ROUNDS=1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r3_h/fetch -o run -- python3 $R/tools/bsr_wave_sweep.py > $R/gpurun_out/r3_h/fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r3_h/write -o run -- python3 $R/tools/bsr_wave_sweep.py > $R/gpurun_out/r3_h/write.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/r3_h/hit -o run -- python3 $R/tools/bsr_wave_sweep.py > $R/gpurun_out/r3_h/hit.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r3_h/ta -o run -- python3 $R/tools/bsr_wave_sweep.py > $R/gpurun_out/r3_h/ta.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/r3_h/sq -o run -- python3 $R/tools/bsr_wave_sweep.py > $R/gpurun_out/r3_h/sq.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum --output-format csv -d $R/gpurun_out/r3_h/tcp -o run -- python3 $R/tools/bsr_wave_sweep.py > $R/gpurun_out/r3_h/tcp.log 2>&1
echo rc=$?
