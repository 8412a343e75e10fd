#!/bin/bash
# LDS bank-conflict attribution for coop3 (run on the GPU box): the default
# build and timing-only variants (tools/build_variant.sh bank_<V> -DC3X_BANK_<V>)
# whose one LDS access pattern is made conflict-free; per build the bench JSON
# line and SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS of the decode kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=${BANK_OUT:-gpurun_out/bank}
mkdir -p $OUT
for v in ${BANK_VARIANTS:-base X MM MST MEM NODMA}; do
    lib=ldpcgputegra_amd/libldpc_mi355x.so
    [ "$v" != base ] && lib=var/variants/bank_$v/libldpc_mi355x.so
    LDPC_MI355X_LIB=$lib timeout -k 10 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-include-regex coop3 \
        -f csv -d $OUT/$v -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $OUT/$v.json 2> $OUT/$v.err
    rc=$?
    echo "$v rc=$rc $(tail -c 300 $OUT/$v.json)" >&2
    [ $rc -ne 0 ] && exit $rc
done
exit 0
