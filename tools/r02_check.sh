#!/bin/bash
# round-2 GPU check: ET / mixed / host-path / shaped-code parity, host-path rates, mixed benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name" >&2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >&2
    tail -4 "gpurun_out/$name.log" >&2
    if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then exit $rc; fi
    return 0
}
[[ ${STEPS:-t} == *t* ]] && step r02_tests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "${TESTK:-early or mixed or host_path or shape}"
[[ ${STEPS:-t} == *h* ]] && step r02_hostrate 300 python tools/host_path_rate.py ${HPCH:-2 1}
[[ ${STEPS:-t} == *m* ]] && step r02_mixed 300 python bench.py --mixed --steps 5 --warmup 2 --cpu-seconds 0
[[ ${STEPS:-t} == *r* ]] && step r02_mixed_ref 300 python bench.py --mixed --mixed-codes reference --steps 5 --warmup 2 --cpu-seconds 0
[[ ${STEPS:-t} == *p* ]] && step r02_mprof 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/mprof -o run -- python3 bench.py --mixed --steps 3 --warmup 1 --cpu-seconds 0
exit 0
