#!/bin/bash
# Same-box A/B of library builds (run on the GPU box): alternates the default
# build and var/variants/<name>/libldpc_mi355x.so, AB_ROUNDS times each, one
# bench.py line per run into $AB_OUT/<name>.jsonl (extra bench args: AB_ARGS).
# A variant "env:VAR=VALUE[,VAR=VALUE]" runs the default build with those
# environment settings instead (runtime switches, no rebuild).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${AB_OUT:-gpurun_out/ab}
mkdir -p $OUT
ARGS=${AB_ARGS:---steps 10 --warmup 2 --cpu-seconds 0}
for i in $(seq ${AB_ROUNDS:-3}); do
    for v in base ${AB_VARIANTS:?}; do
        lib=ldpcgputegra_amd/libldpc_mi355x.so
        envs=()
        case $v in
        base) ;;
        env:*) IFS=, read -r -a envs <<< "${v#env:}" ;;
        *) lib=var/variants/$v/libldpc_mi355x.so ;;
        esac
        f=$OUT/$(echo "$v" | tr ':=,' '___')
        env "${envs[@]}" LDPC_MI355X_LIB=$lib timeout -k 10 150 python3 bench.py $ARGS >> $f.jsonl 2>> $f.err || exit 1
    done
done
for v in base ${AB_VARIANTS}; do
    f=$OUT/$(echo "$v" | tr ':=,' '___')
    python3 -c "
import json,sys
r=[json.loads(l) for l in open('$f.jsonl')]
print('$v', ' '.join('%.3f' % x['roofline']['kernel_ms'] for x in r), 'min %.3f' % min(x['roofline']['kernel_ms'] for x in r))"
done
exit 0
