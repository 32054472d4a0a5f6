#!/bin/bash
# One GPU session: parity tests, the default bench line, a rocprofv3 kernel
# summary of the headline config and the PMC passes bench.py's roofline reads.
# Every GPU step has its own time limit; a crash / timeout stops the session.
#   tools/round_all.sh <tag>
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r02}"
cd "$R" && mkdir -p gpurun_out
PYTHONUNBUFFERED=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.txt; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json | cut -c1-600; echo "bench rc=$rc"
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
[ -n "$NO_PROF" ] && exit 0
PROF_TIMEOUT=300 bash tools/profile.sh > gpurun_out/profile_$TAG.txt 2>&1
rc=$?; tail -8 gpurun_out/profile_$TAG.txt; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_round.sh $TAG
