# round 3, call 2: tile GEMM stamps + debug variants; dequant probe with random zeros; checkpoint test
export TMPDIR=/tmp
O=gpurun_out
TORCHAO_MI355X_LIB=experiments/build/libtilestamps.so timeout -k 10 200 python -u experiments/tile_stamps.py > $O/tile_stamps.jsonl 2> $O/tile_stamps.err && \
timeout -k 10 600 bash experiments/tile_debug.sh run > $O/tile_debug.txt 2>&1 && \
timeout -k 10 200 python -u experiments/probe_aten_dequant_rounding.py --randz > $O/probe_dequant_randz.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_int4.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "reference_written or another_device" > $O/pytest_new2.log 2>&1
