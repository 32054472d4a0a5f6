#!/bin/bash
# Round-5 GPU session.  Every GPU step has its own time limit; a step that
# crashes, aborts or times out ends the session (rc 0 / 1 -- pass / mismatch --
# go on, so a soak that finds wrong answers still lets the rest report).
#   SOAK=1    adapter soaks (tests/cpp suite repeated, tools/diag/copy_soak)
#   TESTS=1   the whole -m gpu suite (no -x: every failure is listed)
#   BENCH=1   bench.py with BENCH_ARGS
#   PROF=1    rocprofv3 kernel-trace stats of the bench
#   OPRATE=1  tools/microbench/oprate4 (VALU issue cost in shader cycles)
#   LISTPMC=1 the counters rocprofv3 offers on this device
#   AB=1      same-process A/B of lib/variants/*.so (tools/exp_variants.py)
#   PMCS=1    stall / issue counters of the pipeline kernels (tools/pmc_stall.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05}
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
    local rc=$?
    tail -8 "gpurun_out/${TAG}_$name.txt"
    echo "== $name rc=$rc"
    if [ $rc -gt 1 ]; then exit $rc; fi
    return 0
}
if [ -n "$SOAK" ]; then
    step suite_repeat 150 tests/cpp/test_dcrt_bin --repeat ${SUITE_REPEAT:-20}
    step modops_repeat 150 tests/cpp/test_dcrt_bin --filter DCRT_mod_ops --repeat ${MODOPS_REPEAT:-5000}
    for v in 0 1 2 3; do
        step copy_soak_v$v 120 tools/diag/copy_soak_bin $v ${SOAK_ITERS:-20000}
    done
fi
if [ -n "$OPRATE" ]; then
    step oprate4 180 tools/microbench/oprate4_bin
fi
if [ -n "$LISTPMC" ]; then
    step pmc_list 120 rocprofv3 --list-avail
fi
if [ -n "$TESTS" ]; then
    PYTHONUNBUFFERED=1 step pytest_gpu 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method=thread ${PYTEST_ARGS}
fi
if [ -n "$AB" ]; then
    EXP_BATCH=${EXP_BATCH:-512} EXP_ROUNDS=${EXP_ROUNDS:-8} step exp_var 300 python -u tools/exp_variants.py
fi
if [ -n "$PMCS" ]; then
    step pmc_stall 600 bash tools/pmc_stall.sh ${TAG}
fi
if [ -n "$BENCH" ]; then
    step bench 400 python -u bench.py ${BENCH_ARGS}
fi
if [ -n "$PROF" ]; then
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py ${BENCH_ARGS}
fi
exit 0
