# round 3 final pass: the default bench line, the kernel-trace profile and the two PMC passes
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_l &&
timeout -k 10 300 python bench.py > gpurun_out/r3_l/bench.json 2> gpurun_out/r3_l/bench.err &&
bash tools/profile_round.sh
