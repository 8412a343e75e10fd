set -o pipefail
mkdir -p gpurun_out/final
O=gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench_default.json 2>&1 && \
timeout -k 10 300 python bench.py --dtype f32 > $O/bench_f32.json 2>&1 && \
timeout -k 10 300 python bench.py --mixed > $O/bench_mixed_b4096.json 2>&1 && \
timeout -k 10 400 python bench.py --mixed --batch 24576 --steps 3 --warmup 1 > $O/bench_mixed_b24576.json 2>&1 && \
timeout -k 10 300 python bench.py --mixed --mixed-codes reference --cpu-seconds 0 > $O/bench_mixed_reference.json 2>&1 && \
for c in "dvbs2_r2_3 2.2" "dvbs2shape_r3_4 2.8" "dvbs2shape_r5_6 3.5" "dvbs2_r8_9 4.6" "dvbs2_r9_10 5.0"; do set -- $c; timeout -k 10 200 python bench.py --code $1 --ebn0 $2 --steps 5 --warmup 1 --cpu-seconds 0 > $O/bench_$1.json 2>&1 || exit 1; done
