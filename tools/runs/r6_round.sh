# Round-6 evidence set on one GPU box: the GPU suite, smoke, the bench line, then the rocprofv3
# kernel-trace / PMC passes of the same bench command (tools/profile_round.sh).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
P=${P:-r06a}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=15 > gpurun_out/${P}_gpu_tests.txt 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1
timeout -k 10 240 python3 bench.py > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err
bash tools/profile_round.sh
