#!/bin/bash
# Round-4 evidence session: the 3,840-case seeded fuzz soak of the GPU path and
# the two-rank gloo rehearsal of the multi-GPU bench on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
OFHE_FUZZ_SCALE=20 timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/fuzz_soak.txt 2>&1
rc=$?; tail -3 gpurun_out/fuzz_soak.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --batch 128 --steps 3 --warmup 1 --ks-batch 2 \
    --ks-steps 3 --c3-batch 64 --cpu-seconds 2 --pcie-chunks 2 > gpurun_out/rehearsal.json 2> gpurun_out/rehearsal.err
rc=$?; tail -c 1500 gpurun_out/rehearsal.json; tail -3 gpurun_out/rehearsal.err; exit $rc
