#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC here; PMC runs
# are separate passes, see tools/pmc.sh).  Output: gpurun_out/prof/
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/prof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof" -o bench -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-extras --no-check \
    ${PROF_ARGS} > "$R/gpurun_out/prof/bench_stdout.json" 2> "$R/gpurun_out/prof/rocprof.err"
rc=$?
echo "rocprof rc=$rc"
find "$R/gpurun_out/prof" -name "*kernel_stats.csv" -exec cat {} \;
exit $rc
