# round 3 start: GPU suite + smoke + bench on the inherited tree
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_a &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_a/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_a/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r3_a/bench.json 2> gpurun_out/r3_a/bench.err
