#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, short bench.  Each GPU step has
# its own time limit; a crash/abort/timeout (rc >= 124) stops the script, an
# ordinary test failure (rc 1) does not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name" >&2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >&2
    tail -5 "gpurun_out/$name.log" >&2
    if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then exit $rc; fi
    return 0
}
STEPS=${STEPS:-smoke,pytest,bench}
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *pytest* ]] && run pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS}
[[ $STEPS == *bench* ]] && run bench 600 python bench.py ${BENCH_ARGS}
if [[ $STEPS == *kernels* ]]; then
    for k in ${KERNELS:-2 3 4}; do
        run bench_k$k 300 python bench.py --kernel $k --steps 3 --warmup 1 --cpu-seconds 0
    done
fi
[[ $STEPS == *sim* ]] && run sim 300 ldpcgputegra_amd/bin/ldpc_sim -code dvbs2_r1_2 -min 0.8 -max 1.2 -pas 0.1 -iter 50 -fer 50 -frames 65536
exit 0
