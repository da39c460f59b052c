# round 3: host cost per sbx_copy in the two tools/capi_overhead modes (tiny fixed copy vs the
# bench's 64 distinct 16^4 slices, short and long loops, small slices), and per-launch BSR n=64
# durations without a profiler (the 14 ms dispatch seen under rocprofv3)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_m && O=gpurun_out/r3_m &&
timeout -k 10 120 tools/capi_overhead > $O/capi_default.txt 2>&1 &&
timeout -k 10 120 tools/capi_overhead permute 16 64 5 > $O/capi_permute.txt 2>&1 &&
timeout -k 10 120 tools/capi_overhead permute 16 64 50 >> $O/capi_permute.txt 2>&1 &&
timeout -k 10 120 tools/capi_overhead permute 4 64 200 >> $O/capi_permute.txt 2>&1 &&
timeout -k 10 120 tools/capi_overhead permute 16 64 5 >> $O/capi_permute.txt 2>&1 &&
timeout -k 10 300 python tools/bsr_outlier.py 3000 64 > $O/bsr_outlier.json 2> $O/bsr_outlier.err
