#!/bin/bash
# Round-4 GPU session for the persistent pipeline (k_pipe): the memory-level
# power probe, the k_pipe parity tests, the same-process A/B against the three
# launches, then (RUN_SUITE=1) the whole GPU suite.  Every GPU step has its own
# time limit; the session stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.txt" 2>&1
    local rc=$?
    tail -15 "gpurun_out/$name.txt"
    echo "== $name rc=$rc"
    return $rc
}
export PYTHONUNBUFFERED=1
if [ -z "$SKIP_POWER" ]; then
    step power_l2 120 bash tools/power_l2.sh || exit $?
fi
step pytest_pipe 300 python -u -m pytest tests/test_gpu_pipe.py -x -v --timeout 200 --timeout-method thread || exit $?
step exp_pipe 300 python -u tools/exp_pipe.py || exit $?
if [ -n "$RUN_SUITE" ]; then
    step pytest_gpu 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread || exit $?
fi
exit 0
