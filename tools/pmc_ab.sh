#!/bin/bash
# PMC passes (tools/profile.sh) for several library builds on one box:
#   VARIANTS="cur var/x/libldpc_mi355x.so" PROF_PASSES="tcpstall tcplat" bash tools/pmc_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for v in ${VARIANTS:-cur}; do
    tag=$(echo "$v" | sed 's#var/##; s#/libldpc_mi355x.so##')
    if [ "$v" = cur ]; then lib=""; else lib="$v"; fi
    LDPC_MI355X_LIB="$lib" PROF_OUT=gpurun_out/pmc_$tag PROF_ARGS="--steps 2 --warmup 1 --cpu-seconds 0" bash tools/profile.sh || exit $?
done
exit 0
