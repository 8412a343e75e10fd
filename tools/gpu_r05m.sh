set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mixed --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r05m_mixed4k.json 2>&1 && \
timeout -k 10 300 python bench.py --mixed --batch 24576 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/r05m_mixed24k.json 2>&1 && \
timeout -k 10 300 python bench.py --mixed --mixed-codes reference --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r05m_mixedref.json 2>&1 && \
LDPC_MI355X_LIB=var/variants/head/libldpc_mi355x.so timeout -k 10 300 python bench.py --mixed --mixed-codes reference --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r05m_mixedref_head.json 2>&1 && \
LDPC_MI355X_LIB=var/variants/head/libldpc_mi355x.so timeout -k 10 300 python bench.py --code dvbs2_r8_9 --ebn0 4.6 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/r05m_r89_head.json 2>&1 && \
LDPC_MI355X_LIB=var/variants/head/libldpc_mi355x.so timeout -k 10 300 python bench.py --code dvbs2shape_r5_6 --ebn0 3.5 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/r05m_r56_head.json 2>&1
