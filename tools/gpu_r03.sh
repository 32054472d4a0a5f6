#!/bin/bash
# Round-3 GPU session steps (each under its own time limit; a crash, abort or
# timeout ends the session, ordinary test failures do not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "== $name" >&2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "rc=$rc" >> "gpurun_out/$name.log"
    echo "$name rc=$rc" >&2
    tail -${TAILN:-15} "gpurun_out/$name.log" >&2
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
for step in ${STEPS}; do
    case $step in
        diag) run diag 120 env T2_ONLY=${T2_ONLY:-2} ./tools/diag/tensor2_asm_diag_bin tools/diag ;;
        m16test) run m16test 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
                    "tests/test_gpu_parity.py::test_block_m16_vs_oracle" ;;
        newtests) run newtests 500 python -u -m pytest -q --timeout 300 --timeout-method thread \
                    tests/test_gpu_headline_shapes.py "tests/test_gpu_rescale.py::test_rescale_rejects_unsafe_aliasing" ;;
        ab) run ab 300 env EXP_CONFIGS="${AB_CONFIGS-;OFHE_BLOCK_M16=1}" EXP_BATCH=${AB_BATCH:-256} EXP_ROUNDS=${AB_ROUNDS:-6} \
                    python -u tools/exp_variants.py ;;
        ks) run ks 400 env EXP_TOGGLE="${KS_TOGGLE}" EXP_ROUNDS=${KS_ROUNDS:-8} EXP_ONLY=${KS_ONLY:-libofhe_hip_floor} \
                    python -u tools/exp_ks.py ;;
        suite) run suite 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ;;
        bench) run bench 400 python bench.py ${BENCH_ARGS} ;;
        pmcm16) run pmcm16 300 env OFHE_BLOCK_M16=1 ./tools/pmc_m16.sh && run pmck16 300 env OFHE_BLOCK_M16=0 ./tools/pmc_m16.sh ;;
        *) echo "unknown step $step" >&2; exit 2 ;;
    esac
done
