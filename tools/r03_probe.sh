#!/bin/bash
# round-3 GPU session runner: each step has its own time limit; a crash /
# abort / timeout (rc >= 124, or any rc > 1 but 5) stops the script, an
# ordinary test failure (rc 1) does not.  Steps (STEPS, comma list):
#   valu    tools/ubench_valu        VALU issue rates
#   vmem    tools/ubench_vmem        coop3's vector-memory pattern, floors
#   bench   bench.py (default workload, short)
#   tests   pytest -m gpu (TESTS: files / -k filter via PYTEST_ARGS)
#   prof    tools/profile.sh passes (PROF_PASSES)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03}
mkdir -p "$OUT"
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >&2
    tail -4 "$OUT/$name.log" >&2
    if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then exit $rc; fi
    return 0
}
STEPS=${STEPS:-bench}
for s in ${STEPS//,/ }; do
    case $s in
    valu) step ubench_valu 60 ./tools/ubench_valu ;;
    vmem) step ubench_vmem 120 ./tools/ubench_vmem ldpcgputegra_amd/codes/dvbs2_r1_2.txt ;;
    lc) step ubench_lc 120 ./tools/ubench_lc ;;
    bench) step bench 300 python3 bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --cpu-seconds 0} ;;
    mixed) step bench_mixed 300 python3 bench.py --mixed ${BENCH_ARGS:---steps 5 --warmup 2 --cpu-seconds 0} ;;
    tests) step tests 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "${TESTK:-not nothing}" ;;
    prof) PROF_OUT=$OUT/prof bash tools/profile.sh || exit $? ;;
    hostrate) step host_rate 300 python3 tools/host_path_rate.py ${HOST_CHUNKS:-2 1} ;;
    hptrace) step host_trace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/hptrace" -o hp -- python3 tools/host_path_rate.py 2 ;;
    smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    esac
done
exit 0
