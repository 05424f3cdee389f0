# round 3 (re-entry), call 2: bench after the fence-gate fix; L2 intake probe; tile GEMM stamps and
# timing-only variants (why the LDS-DMA tile kernel loses to gemm_mfma at M = 128)
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-reference-gpu > $O/bench_r3b.json 2> $O/bench_r3b.err && \
timeout -k 10 120 ./experiments/build/probe_l2_intake > $O/probe_l2_intake.jsonl 2>&1 && \
TORCHAO_MI355X_LIB=experiments/build/libtilestamps.so timeout -k 10 200 python -u experiments/tile_stamps.py > $O/tile_stamps.jsonl 2> $O/tile_stamps.err && \
timeout -k 10 600 bash experiments/tile_debug.sh run > $O/tile_debug.txt 2>&1
