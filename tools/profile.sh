#!/bin/bash
# rocprofv3 collection for the bench workload (run on the GPU box).
#   pass "trace": --kernel-trace --stats         -> per-kernel durations (+ the bench JSON line)
#   pass "fetch": --pmc FETCH_SIZE               -> HBM read bytes (KB; gfx950 counts 1/2 of wide reads)
#   pass "write": --pmc WRITE_SIZE               -> HBM write bytes (KB)
#   pass "sq":    wave-state counters            -> issue vs wait breakdown
#   pass "tcc":   L2 hit / miss
# Counters get their own passes, filtered to the decode kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
# the trace pass runs >= 10 measured launches after 2 warm-up ones (tools/
# summarize_profiles.py drops the warm-up launches and reports the median);
# counter passes replay every dispatch, so they run a short bench
TARGS=${PROF_TRACE_ARGS:---steps 12 --warmup 2 --cpu-seconds 0}
ARGS=${PROF_ARGS:---steps 3 --warmup 1 --cpu-seconds 0}
KRE=${PROF_KERNEL_RE:-decode}
PASSES=${PROF_PASSES:-trace fetch write sq tcc}
run() {
    local name=$1 secs=$2
    shift 2
    echo "== $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >&2
    tail -3 "$OUT/$name.log" >&2
    [ $rc -ne 0 ] && exit $rc
    return 0
}
for p in $PASSES; do
    case $p in
    trace) run trace 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py $TARGS ;;
    fetch) run fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/fetch -o run -- python3 bench.py $ARGS ;;
    write) run write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/write -o run -- python3 bench.py $ARGS ;;
    sq) run sq 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-include-regex "$KRE" -f csv -d $OUT/sq -o run -- python3 bench.py $ARGS ;;
    sq2) run sq2 600 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES --kernel-include-regex "$KRE" -f csv -d $OUT/sq2 -o run -- python3 bench.py $ARGS ;;
    tlb) run tlb 600 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_REQUEST TCP_UTCL1_STALL_MULTI_MISS --kernel-include-regex "$KRE" -f csv -d $OUT/tlb -o run -- python3 bench.py $ARGS ;;
    tcplat) run tcplat 600 rocprofv3 --pmc TCP_TCC_WRITE_REQ_LATENCY TCP_TCC_READ_REQ_LATENCY TCP_TCC_WRITE_REQ TCP_TCC_READ_REQ TA_ADDR_STALLED_BY_TC_CYCLES TA_BUSY --kernel-include-regex "$KRE" -f csv -d $OUT/tcplat -o run -- python3 bench.py $ARGS ;;
    tcpstall) run tcpstall 600 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_UTCL1_SERIALIZATION_STALL TA_DATA_STALLED_BY_TC_CYCLES TA_TA_BUSY --kernel-include-regex "$KRE" -f csv -d $OUT/tcpstall -o run -- python3 bench.py $ARGS ;;
    # configs[4]: PMC over every kernel of the step (tools/mixed_traffic.py: MIX_ARGS e.g. --batch 24576)
    mixfetch) run mixfetch 600 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/mixfetch -o run -- python3 bench.py --mixed $ARGS ${MIX_ARGS:-} ;;
    mixwrite) run mixwrite 600 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/mixwrite -o run -- python3 bench.py --mixed $ARGS ${MIX_ARGS:-} ;;
    mixtrace) run mixtrace 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/mixtrace -o run -- python3 bench.py --mixed $TARGS ${MIX_ARGS:-} ;;
    list) timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true ;;
    tcc) run tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KRE" -f csv -d $OUT/tcc -o run -- python3 bench.py $ARGS ;;
    esac
done
exit 0
