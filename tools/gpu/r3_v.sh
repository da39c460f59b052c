# round 3 (session 2): the default bench line, the kernel-trace profile and the two PMC passes on
# the tree with the site-block transpose kernel
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_v &&
timeout -k 10 300 python bench.py > gpurun_out/r3_v/bench.json 2> gpurun_out/r3_v/bench.err &&
bash tools/profile_round.sh
