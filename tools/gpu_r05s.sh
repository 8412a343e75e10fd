set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_coop3_r23.py -x -q --timeout 200 --timeout-method thread -k "fixed or early or nms" > gpurun_out/r05s_tests.txt 2>&1 && \
AB_OUT=gpurun_out/r05s_ab910 AB_VARIANTS=nopre AB_ROUNDS=2 AB_ARGS="--code dvbs2_r9_10 --ebn0 5.0 --steps 4 --warmup 1 --cpu-seconds 0" timeout -k 10 300 bash tools/ab_lib.sh && \
AB_OUT=gpurun_out/r05s_ab34 AB_VARIANTS=nopre AB_ROUNDS=2 AB_ARGS="--code dvbs2shape_r3_4 --ebn0 2.8 --steps 5 --warmup 1 --cpu-seconds 0" timeout -k 10 300 bash tools/ab_lib.sh && \
AB_OUT=gpurun_out/r05s_ab12 AB_VARIANTS="chunk5 head" AB_ROUNDS=3 timeout -k 10 600 bash tools/ab_lib.sh
