#!/bin/bash
# coop3 (kernel 8) diagnostics on the GPU box:
#   tools/coop3_diag.sh parity            GPU parity subset (golden, DVB-S2 full batch, early termination)
#   tools/coop3_diag.sh stamps            per-phase cycle stamps (diagnostic build path) + kernel time
#   tools/coop3_diag.sh variants v...     stamps + kernel time of build/variants/<v> (tools/build_variant.sh)
#   tools/coop3_diag.sh pmc "<passes>" [v...]   tools/profile.sh passes for the default library and variants
#   tools/coop3_diag.sh ws                stamps at WS = 3 and 4 slab waves
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --kernel 8 --cpu-seconds 0"
stamps() {  # stamps <lib or ''>
    LDPC_MI355X_LIB=$1 LDPC_COOP3_STAMP=1 timeout -k 10 200 $B --steps 1 --warmup 0 > gpurun_out/c3_s.log 2>&1 || exit 1
    grep -A8 stamps gpurun_out/c3_s.log
    LDPC_MI355X_LIB=$1 timeout -k 10 200 $B --steps 5 --warmup 1 > gpurun_out/c3_b.log 2>&1 || exit 1
    grep -o '"kernel_ms": [0-9.]*' gpurun_out/c3_b.log
}
cmd=$1
shift
case $cmd in
parity)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
        --timeout-method thread -k "golden or dvbs2 or coop2_early" > gpurun_out/c3_pytest.log 2>&1
    rc=$?
    tail -3 gpurun_out/c3_pytest.log
    exit $rc ;;
stamps) stamps "" ;;
variants) for v in "$@"; do echo "== $v"; stamps build/variants/$v/libldpc_mi355x.so; done ;;
ws)
    for ws in 3 4; do
        echo "== WS $ws"
        LDPC_COOP3_WS=$ws LDPC_COOP3_STAMP=1 timeout -k 10 200 $B --steps 1 --warmup 0 > gpurun_out/c3_s.log 2>&1 || exit 1
        grep -A8 stamps gpurun_out/c3_s.log
    done ;;
pmc)
    P=$1
    shift
    A="--kernel 8 --steps 2 --warmup 1 --cpu-seconds 0"
    PROF_OUT=gpurun_out/prof PROF_ARGS="$A" PROF_KERNEL_RE=coop3_decode PROF_PASSES="$P" bash tools/profile.sh || exit 1
    for v in "$@"; do
        LDPC_MI355X_LIB=build/variants/$v/libldpc_mi355x.so PROF_OUT=gpurun_out/prof_$v PROF_ARGS="$A" \
            PROF_KERNEL_RE=coop3_decode PROF_PASSES="$P" bash tools/profile.sh || exit 1
    done ;;
*) echo "unknown command $cmd" >&2; exit 2 ;;
esac
