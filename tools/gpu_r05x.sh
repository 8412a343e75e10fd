set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "error_counter or decode_count or full_batch or golden" > gpurun_out/r05x_tests.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r05x_trace -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/r05x_trace.log 2>&1
