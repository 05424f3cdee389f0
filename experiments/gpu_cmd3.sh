# round 3, call 3: LDS-DMA tile GEMM: tests, A/B, stamps, debug variants
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_tile.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_tile5.log 2>&1 && \
timeout -k 10 300 python -u experiments/ab_tile.py --quick > $O/ab_tile5.jsonl 2> $O/ab_tile5.err && \
TORCHAO_MI355X_LIB=experiments/build/libtilestamps.so timeout -k 10 200 python -u experiments/tile_stamps.py > $O/tile_stamps5.jsonl 2> $O/tile_stamps5.err && \
timeout -k 10 600 bash experiments/tile_debug.sh run > $O/tile_debug5.txt 2>&1
