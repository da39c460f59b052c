# round 3: permute slice micro (kernel-argument size effect)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_s && O=gpurun_out/r3_s &&
timeout -k 10 120 tools/permute_micro > $O/permute_micro2.txt 2>&1
