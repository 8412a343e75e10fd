set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coop3_r23.py -x -q --timeout 200 --timeout-method thread -k "test_gpu_matches_reference_golden or test_dvbs2_full_batch_vs_reference or test_early_termination_vs_oracle or fixed_iterations or nms_fixed" > gpurun_out/r05n_tests.txt 2>&1 && \
AB_OUT=gpurun_out/r05n_ab AB_VARIANTS="xo8 head" AB_ROUNDS=3 timeout -k 10 700 bash tools/ab_lib.sh
