#!/bin/bash
# GPU-box check sequence: parity tests, then smoke.  Each GPU step has its own
# time limit; anything other than a clean pass/fail (0/1) stops the sequence.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${GZ_TEST_TIMEOUT:-900} python -m pytest tests/test_gpu.py -q -p no:cacheprovider \
  --timeout 600 -rf ${GZ_PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a gpurun_out/gpu_tests.log
tail -40 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
echo "smoke rc=$src"; tail -5 gpurun_out/smoke.log
exit $(( rc != 0 ? rc : src ))
