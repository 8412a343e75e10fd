set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_coop3_r23.py -x -q --timeout 200 --timeout-method thread -k "(r5_6 or r8_9 or r9_10)" > gpurun_out/r05t_tests.txt 2>&1 && \
AB_OUT=gpurun_out/r05t_ab910 AB_VARIANTS=postfirst AB_ROUNDS=2 AB_ARGS="--code dvbs2_r9_10 --ebn0 5.0 --steps 4 --warmup 1 --cpu-seconds 0" timeout -k 10 300 bash tools/ab_lib.sh && \
AB_OUT=gpurun_out/r05t_ab56 AB_VARIANTS=postfirst AB_ROUNDS=2 AB_ARGS="--code dvbs2shape_r5_6 --ebn0 3.5 --steps 4 --warmup 1 --cpu-seconds 0" timeout -k 10 300 bash tools/ab_lib.sh && \
LDPC_COOP3_STAMP=1 timeout -k 10 200 python bench.py --code dvbs2_r9_10 --ebn0 5.0 --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/r05t_stamps_r910.txt 2>&1
