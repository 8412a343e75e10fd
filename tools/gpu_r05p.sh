set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_coop3_r23.py -x -q --timeout 200 --timeout-method thread -k "(r5_6 or r8_9 or r9_10) and (fixed or early)" > gpurun_out/r05p_tests.txt 2>&1 && \
for c in "dvbs2shape_r5_6 3.5" "dvbs2_r8_9 4.6" "dvbs2_r9_10 5.0"; do set -- $c; timeout -k 10 200 python bench.py --code $1 --ebn0 $2 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/r05p_$1.json 2>&1 || exit 1; done && \
LDPC_COOP3_STAMP=1 timeout -k 10 200 python bench.py --code dvbs2_r9_10 --ebn0 5.0 --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/r05p_stamps_r910.txt 2>&1
