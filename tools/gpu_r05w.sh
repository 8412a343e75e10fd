set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coop3_r23.py tests/test_gpu_configs4.py -x -q --timeout 200 --timeout-method thread -k "golden or soft_output or full_batch or node_major or fixed_iterations or as_benched" > gpurun_out/r05w_tests.txt 2>&1 && \
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r05w_bench.json 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r05w_trace -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/r05w_trace.log 2>&1
