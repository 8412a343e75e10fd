#!/bin/bash
# Same-box A/B of library builds on the default bench workload (box-to-box
# spread is ~5 %, larger than most kernel changes).  Run on the GPU box:
#   VARIANTS="cur var/base/libldpc_mi355x.so ..." ROUNDS=2 bash tools/ab.sh
# "cur" = the in-tree library.  Prints one line per run: variant, kernel_ms,
# ms_per_step.  Extra env per run: AB_ENV (e.g. LDPC_COOP3_STAMP=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
ARGS=${AB_ARGS:---steps 10 --warmup 2 --cpu-seconds 0}
i=0
for r in $(seq 1 "${ROUNDS:-2}"); do
    for v in ${VARIANTS:-cur}; do
        i=$((i + 1))
        if [ "$v" = cur ]; then lib=""; else lib="$v"; fi
        LDPC_MI355X_LIB="$lib" LDPC_AB_OLD_LIB=1 timeout -k 10 240 env $AB_ENV python3 bench.py $ARGS > "$OUT/run$i.log" 2>&1
        rc=$?
        if [ $rc -ne 0 ]; then
            echo "$v rc=$rc"
            tail -5 "$OUT/run$i.log"
            exit $rc
        fi
        python3 - "$v" "$OUT/run$i.log" <<'EOF'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d = json.loads(line)
        print("%-40s kernel_ms %.3f step_ms %.3f" % (sys.argv[1], d["roofline"]["kernel_ms"], d["ms_per_step"]))
EOF
    done
done
exit 0
