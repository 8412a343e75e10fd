set -o pipefail
mkdir -p gpurun_out
AB_OUT=gpurun_out/r05y_ab12 AB_VARIANTS="bprio1 msl6 msl2" AB_ROUNDS=3 timeout -k 10 900 bash tools/ab_lib.sh
