#!/bin/bash
# Measurement session: bench line, rocprofv3 kernel stats, PMC passes for
# profiles/pmc_current.json.  Each GPU step under its own time limit.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r04}"
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 400 python3 -u bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
PROF_TIMEOUT=300 bash tools/profile.sh > gpurun_out/prof_$TAG.txt 2>&1
rc=$?; tail -8 gpurun_out/prof_$TAG.txt; [ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_PMC" ]; then
    bash tools/pmc_round.sh $TAG > gpurun_out/pmc_$TAG.log 2>&1
    rc=$?; tail -30 gpurun_out/pmc_$TAG.log; exit $rc
fi
