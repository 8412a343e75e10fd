#!/bin/bash
# One parametrised GPU-box session (replaces the per-round one-off scripts).
#   TAG=r06a STEPS="tests bench f32 mixed" bash tools/gpu_session.sh
# Every step runs under its own time limit, output to gpurun_out/$TAG/<step>.*;
# a crash / abort / time limit (rc >= 124) or any failure stops the session
# (no later GPU step runs after a fault).  Steps:
#   smoke      __graft_entry__.smoke()
#   tests      pytest -m gpu (PYTEST_K: -k filter; PYTEST_FILES: files, default tests)
#   bench      bench.py, configs[2] default line (BENCH_ARGS extra)
#   f32        bench.py --dtype f32 (configs[1])
#   mixed      bench.py --mixed (configs[4], batch 4096)
#   mixed24k   bench.py --mixed --batch 24576
#   mixedref   bench.py --mixed --mixed-codes reference
#   codes      bench.py per DVB-S2 code (CODES: "code:ebn0 ..."), fixed 50 it
#   stamps     LDPC_COOP3_STAMP=1 cycle stamps per code (STAMP_CODES: "code:ebn0 ...")
#   ab         tools/ab_lib.sh (AB_VARIANTS, AB_ARGS, AB_ROUNDS)
#   prof       tools/profile.sh (PROF_PASSES, PROF_ARGS, MIX_ARGS) into gpurun_out/$TAG/prof
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-session}
O=gpurun_out/$TAG
mkdir -p "$O"
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name" >&2
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >&2
    tail -4 "$O/$name.log" >&2
    [ $rc -ne 0 ] && exit $rc
    return 0
}
CODES=${CODES:-"dvbs2_r2_3:2.2 dvbs2shape_r3_4:2.8 dvbs2shape_r5_6:3.5 dvbs2_r8_9:4.6 dvbs2_r9_10:5.0"}
for s in ${STEPS:-smoke tests bench}; do
    case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 1100 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q -p no:cacheprovider --timeout 200 \
               --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ;;
    bench) step bench 300 python bench.py ${BENCH_ARGS:-} ;;
    f32) step f32 300 python bench.py --dtype f32 ${BENCH_ARGS:-} ;;
    mixed) step mixed 300 python bench.py --mixed ${BENCH_ARGS:-} ;;
    mixed24k) step mixed24k 400 python bench.py --mixed --batch 24576 --steps 3 --warmup 1 ${BENCH_ARGS:-} ;;
    mixedref) step mixedref 300 python bench.py --mixed --mixed-codes reference --cpu-seconds 0 ;;
    codes) for c in $CODES; do
               step "code_${c%%:*}" 200 python bench.py --code ${c%%:*} --ebn0 ${c##*:} --steps 5 --warmup 1 --cpu-seconds 0
           done ;;
    stamps) for c in ${STAMP_CODES:-dvbs2_r1_2:1.0}; do
               step "stamps_${c%%:*}" 200 env LDPC_COOP3_STAMP=1 python bench.py --code ${c%%:*} --ebn0 ${c##*:} --steps 1 \
                   --warmup 0 --cpu-seconds 0
            done ;;
    ab) step ab 1000 env AB_OUT=$O/ab bash tools/ab_lib.sh ;;
    prof) step prof 1100 env PROF_OUT=$O/prof bash tools/profile.sh ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
    esac
done
exit 0
