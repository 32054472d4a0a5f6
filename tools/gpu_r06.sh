#!/bin/bash
# Round-6 GPU session.  Every GPU step has its own time limit; a step that
# crashes, aborts or times out ends the session (rc 0 / 1 -- pass / mismatch --
# go on, so a red check still lets the rest report).
#   HOOKS=1   tests/cpp/test_hooks_bin (hook bodies, both gate branches, KS hook)
#   XOVER=1   tests/cpp/hook_crossover_bin (the gate's measured table)
#   CHAIN=1   tests/cpp/chain_bin timing (adapter chain, per-chain ms)
#   TESTS=1   the whole -m gpu suite (no -x: every failure is listed)
#   BENCH=1   bench.py with BENCH_ARGS
#   PROF=1    rocprofv3 kernel-trace stats of the headline bench (tools/profile.sh)
#   PMC=1     the PMC passes bench.py's roofline reads (tools/pmc_round.sh)
#   AB=1      same-process A/B of lib/variants/*.so (tools/exp_variants.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
    local rc=$?
    tail -${TAILN:-8} "gpurun_out/${TAG}_$name.txt"
    echo "== $name rc=$rc"
    if [ $rc -gt 1 ]; then exit $rc; fi
    return 0
}
if [ -n "$HOOKS" ]; then
    step hooks 120 tests/cpp/test_hooks_bin gpurun_out/${TAG}_ks_hook.bin
fi
if [ -n "$XOVER" ]; then
    OMP_NUM_THREADS=${OMP_NUM_THREADS:-16} TAILN=14 step crossover 420 tests/cpp/hook_crossover_bin ${XOVER_ARGS}
fi
if [ -n "$CHAIN" ]; then
    step chain 120 tests/cpp/chain_bin gpurun_out/${TAG}_chain.bin 20
fi
if [ -n "$TESTS" ]; then
    PYTHONUNBUFFERED=1 step pytest_gpu 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method=thread ${PYTEST_ARGS}
fi
if [ -n "$AB" ]; then
    EXP_BATCH=${EXP_BATCH:-512} EXP_ROUNDS=${EXP_ROUNDS:-8} step exp_var 300 python -u tools/exp_variants.py
fi
if [ -n "$BENCH" ]; then
    TAILN=2 step bench 400 python -u bench.py ${BENCH_ARGS}
fi
if [ -n "$PROF" ]; then
    PROF_TIMEOUT=300 step prof 330 bash tools/profile.sh
fi
if [ -n "$PMC" ]; then
    step pmc 900 bash tools/pmc_round.sh ${TAG}
fi
exit 0
