set -o pipefail
mkdir -p gpurun_out
AB_OUT=gpurun_out/r05v_ab56 AB_VARIANTS="pc8 pc2 msl0" AB_ROUNDS=2 AB_ARGS="--code dvbs2shape_r5_6 --ebn0 3.5 --steps 4 --warmup 1 --cpu-seconds 0" timeout -k 10 500 bash tools/ab_lib.sh && \
AB_OUT=gpurun_out/r05v_ab910 AB_VARIANTS="pc8 pc2 msl0" AB_ROUNDS=2 AB_ARGS="--code dvbs2_r9_10 --ebn0 5.0 --steps 4 --warmup 1 --cpu-seconds 0" timeout -k 10 500 bash tools/ab_lib.sh && \
AB_OUT=gpurun_out/r05v_ab23 AB_VARIANTS="pc8 pc2" AB_ROUNDS=2 AB_ARGS="--code dvbs2_r2_3 --ebn0 2.2 --steps 4 --warmup 1 --cpu-seconds 0" timeout -k 10 400 bash tools/ab_lib.sh
