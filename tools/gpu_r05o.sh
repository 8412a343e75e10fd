set -o pipefail
mkdir -p gpurun_out
LDPC_COOP3_STAMP=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/r05o_stamps_r12.txt 2>&1 && \
LDPC_COOP3_STAMP=1 timeout -k 10 200 python bench.py --code dvbs2_r9_10 --ebn0 5.0 --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/r05o_stamps_r910.txt 2>&1 && \
LDPC_COOP3_STAMP=1 timeout -k 10 200 python bench.py --code dvbs2shape_r5_6 --ebn0 3.5 --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/r05o_stamps_r56.txt 2>&1 && \
timeout -k 10 300 python bench.py --mixed --batch 24576 --steps 3 --warmup 1 > gpurun_out/r05o_mixed24k_cpu.json 2>&1
