# round 3: the whole -m gpu suite and smoke on the tree with the site-block transpose kernel
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_t && O=gpurun_out/r3_t &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
