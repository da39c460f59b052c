# round 3: one-wave-per-row 3x3 BSR kernel vs the existing forms, by rhs columns
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_g &&
timeout -k 10 300 python tools/bsr_wave_sweep.py > gpurun_out/r3_g/sweep_z.json 2> gpurun_out/r3_g/sweep_z.err &&
DTYPE=complex64 NS=12,32,64,128 FORMS=default,row_chunk,wave_pd1,wave_pd2,wave_pd4 timeout -k 10 300 python tools/bsr_wave_sweep.py > gpurun_out/r3_g/sweep_c.json 2> gpurun_out/r3_g/sweep_c.err
