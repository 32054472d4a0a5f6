#!/bin/bash
# Round-4 ICOL next-source prefetch: key-switch parity on the new build, then
# the same-process A/B of OFHE_BCC_PREF=0 / 1 (lib/variants) on configs[4].
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_keyswitch.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_ks_pref.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_ks_pref.txt; [ $rc -eq 0 ] || exit $rc
EXP_ROUNDS=9 timeout -k 10 300 python -u tools/exp_ks.py > gpurun_out/pref_ab.txt 2>&1
rc=$?; tail -12 gpurun_out/pref_ab.txt; exit $rc
