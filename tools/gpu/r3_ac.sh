# round 3 (session 2): run-to-run determinism of the 12x12 block-staged BSR kernel
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_ac && O=gpurun_out/r3_ac &&
timeout -k 10 300 python tools/bsr_determinism.py > $O/det.txt 2> $O/det.err
