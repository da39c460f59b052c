# round 3: the default bench line on the tree with both transpose kernels
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_x &&
timeout -k 10 300 python bench.py > gpurun_out/r3_x/bench.json 2> gpurun_out/r3_x/bench.err
