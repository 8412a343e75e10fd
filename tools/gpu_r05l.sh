set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_coop3_r23.py -x -v --timeout 200 --timeout-method thread -k "r5_6 or r8_9 or r9_10" > gpurun_out/r05l_tests.txt 2>&1 && \
for c in "dvbs2shape_r5_6 3.5" "dvbs2_r8_9 4.6" "dvbs2_r9_10 5.0"; do set -- $c; for k in 8 0; do timeout -k 10 200 python bench.py --code $1 --ebn0 $2 --kernel $k --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/r05l_$1_k$k.json 2>&1 || exit 1; done; done && \
AB_OUT=gpurun_out/r05l_ab AB_VARIANTS=head AB_ROUNDS=3 timeout -k 10 500 bash tools/ab_lib.sh
