# round 3: multi-tile pipelined copy kernel -- correctness, then the config-2p slice loop sweep
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_i &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_copy.py -q --timeout 200 --timeout-method thread > gpurun_out/r3_i/tests.log 2>&1 &&
timeout -k 10 300 python tools/permute_sweep.py > gpurun_out/r3_i/sweep.json 2> gpurun_out/r3_i/sweep.err
