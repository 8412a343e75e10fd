set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_coop3_r23.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "r2_3 or r3_4 or test_gpu_matches_reference_golden or test_early_termination_vs_oracle or staged" > gpurun_out/r05u_tests.txt 2>&1 && \
AB_OUT=gpurun_out/r05u_ab23 AB_VARIANTS=pf1 AB_ROUNDS=2 AB_ARGS="--code dvbs2_r2_3 --ebn0 2.2 --steps 5 --warmup 1 --cpu-seconds 0" timeout -k 10 300 bash tools/ab_lib.sh && \
AB_OUT=gpurun_out/r05u_ab34 AB_VARIANTS=pf1 AB_ROUNDS=2 AB_ARGS="--code dvbs2shape_r3_4 --ebn0 2.8 --steps 5 --warmup 1 --cpu-seconds 0" timeout -k 10 300 bash tools/ab_lib.sh && \
AB_OUT=gpurun_out/r05u_ab12 AB_VARIANTS="pf3" AB_ROUNDS=3 timeout -k 10 400 bash tools/ab_lib.sh && \
LDPC_MI355X_LIB=var/variants/pf3/libldpc_mi355x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "test_gpu_matches_reference_golden and r1_2" > gpurun_out/r05u_pf3_tests.txt 2>&1
