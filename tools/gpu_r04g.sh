#!/bin/bash
# Power probe of the persistent pipeline against the three launches (batch 1024)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PS_BATCH=1024
bash tools/power_probe.sh three all 8 || exit $?
PS_PIPE=12 bash tools/power_probe.sh pipe12 all 8 || exit $?
PS_PIPE=12 OFHE_PIPE_SC1=1 bash tools/power_probe.sh pipe12s all 8 || exit $?
