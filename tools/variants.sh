#!/bin/bash
# Bench variants on the GPU box: each argument is NAME:ENV1=V1,ENV2=V2 ...
# (environment knobs of the decoder), run as a short bench (and a stamped
# bench when STAMP=1) with its own time limit; stops at the first crash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/var
ARGS=${VAR_ARGS:---steps 5 --warmup 1 --cpu-seconds 0}
for spec in "$@"; do
    name=${spec%%:*}
    envs=${spec#*:}
    [ "$envs" = "$spec" ] && envs=""
    (
        IFS=',' read -ra kvs <<< "$envs"
        for kv in "${kvs[@]}"; do [ -n "$kv" ] && export "$kv"; done
        timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/var/$name.log 2>&1 || exit $?
        if [ "${STAMP:-0}" = 1 ]; then
            LDPC_COOP2_STAMP=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 \
                > gpurun_out/var/${name}_stamp.log 2>&1 || exit $?
        fi
    ) || { echo "variant $name failed rc=$?"; exit 1; }
    python3 - "$name" <<'PY'
import json, sys
name = sys.argv[1]
for suffix in ("", "_stamp"):
    try:
        lines = open("gpurun_out/var/%s%s.log" % (name, suffix)).read().splitlines()
    except OSError:
        continue
    for l in lines:
        if l.startswith("coop2 stamps"):
            print(name, l)
        if l.startswith("{") and not suffix:
            j = json.loads(l)
            print("%-16s %9.1f Mbit/s  kernel %.3f ms  frac %.3f" % (name, j["value"], j["roofline"]["kernel_ms"], j["roofline"]["frac"]))
PY
done
exit 0
