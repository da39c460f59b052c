# round 3 (session 2): full suite on the tree after the fuzz fixes
# the two PMC passes on the tree with both transpose kernels
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_ao && O=gpurun_out/r3_ao &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
bash tools/profile_round.sh
