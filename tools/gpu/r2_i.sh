cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2_chain_test.log 2>&1 ;
bash tools/profile_round.sh
