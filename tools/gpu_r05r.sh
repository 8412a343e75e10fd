set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_coop3_r23.py -x -q --timeout 200 --timeout-method thread -k "(r2_3 or r3_4) and (fixed or early or nms)" > gpurun_out/r05r_tests.txt 2>&1 && \
AB_OUT=gpurun_out/r05r_ab23 AB_VARIANTS=chunk20 AB_ROUNDS=2 AB_ARGS="--code dvbs2_r2_3 --ebn0 2.2 --steps 5 --warmup 1 --cpu-seconds 0" timeout -k 10 400 bash tools/ab_lib.sh && \
AB_OUT=gpurun_out/r05r_ab34 AB_VARIANTS=chunk20 AB_ROUNDS=2 AB_ARGS="--code dvbs2shape_r3_4 --ebn0 2.8 --steps 5 --warmup 1 --cpu-seconds 0" timeout -k 10 400 bash tools/ab_lib.sh
