#!/bin/bash
# One GPU session: parity tests, then (only if no crash/timeout) the bench.
# Exit codes 0/1 from pytest (pass / test failures) allow the bench; anything
# else (abort, segfault, timeout) stops the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTHONUNBUFFERED=1 timeout -k 10 ${PYTEST_TIMEOUT:-500} python -m pytest ${PYTEST_PATHS:-tests} -m gpu -q -rf --timeout 240 --timeout-method=thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.txt
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
echo "bench rc=$brc"
exit $brc
