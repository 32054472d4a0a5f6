#!/bin/bash
# Round-4 GPU session: GPU parity suite on the default build, then same-process
# A/B of the variant builds (pipeline and key switch).  Every GPU step has its
# own time limit; the session stops at the first crash / timeout.
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
if [ -z "$SKIP_TESTS" ]; then
    PYTHONUNBUFFERED=1 step pytest_gpu 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method=thread ${PYTEST_ARGS}
    rc=$?
    if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -z "$SKIP_AB" ]; then
    EXP_BATCH=${EXP_BATCH:-512} EXP_ROUNDS=${EXP_ROUNDS:-8} step exp_var 300 python -u tools/exp_variants.py || exit $?
    if [ -z "$SKIP_KS" ]; then
        EXP_ROUNDS=${EXP_KS_ROUNDS:-6} step exp_ks 300 python -u tools/exp_ks.py || exit $?
    fi
fi
if [ -n "$RUN_DIAG" ]; then
    # VGPR-allocation sweep of the round-2 EvalMultCore machine code
    T2_SWEEP=1 step vgpr_sweep 180 tools/diag/tensor2_asm_diag_bin tools/diag || exit $?
fi
if [ -n "$RUN_BENCH" ]; then
    step bench 400 python -u bench.py ${BENCH_ARGS} || exit $?
fi
exit 0
