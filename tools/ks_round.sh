#!/bin/bash
# Key-switch (configs[4]) bench line + rocprofv3 kernel stats of it.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/ksprof"
cd "$R"
timeout -k 10 300 python3 bench.py --workload keyswitch --steps ${KS_STEPS:-10} --warmup 2 ${KS_ARGS} > gpurun_out/ks_bench.json 2> gpurun_out/ks_bench.err
rc=$?; cat gpurun_out/ks_bench.json; tail -3 gpurun_out/ks_bench.err; echo "ks bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ksprof" -o ks -- python3 "$R/bench.py" --workload keyswitch --steps 3 --warmup 1 ${KS_ARGS} > "$R/gpurun_out/ksprof/stdout.json" 2> "$R/gpurun_out/ksprof/rocprof.err"
rc=$?
echo "rocprof rc=$rc"
find "$R/gpurun_out/ksprof" -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
exit $rc
