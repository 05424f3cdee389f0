# round 3, call 1: probes (aten dequant rounding, L2 intake), the new/changed GPU tests, tile GEMM A/B
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 ./experiments/build/probe_l2_intake > $O/probe_l2_intake.jsonl 2>&1 && \
timeout -k 10 300 python -u experiments/probe_aten_dequant_rounding.py > $O/probe_dequant.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_tile.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_tile.log 2>&1 && \
timeout -k 10 300 python -u experiments/ab_tile.py --quick > $O/ab_tile_quick.jsonl 2> $O/ab_tile_quick.err && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_int4.py tests/test_gpu_int8.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "aten or reference_written or another_device or intmm or int_scaled or safe_int" > $O/pytest_new1.log 2>&1
