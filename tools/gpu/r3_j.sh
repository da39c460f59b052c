# round 3: direct (destination-ordered) copy kernel vs the LDS-tiled one on the config-2p slices
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_j &&
timeout -k 10 300 python tools/permute_sweep.py > gpurun_out/r3_j/sweep.json 2> gpurun_out/r3_j/sweep.err
