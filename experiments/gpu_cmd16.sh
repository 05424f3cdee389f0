# round 3, call 8: stream GEMM parity tests, A/B against the previous routing, GEMM test files
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_gemm_stream.py > $O/pytest_stream.log 2>&1 && \
timeout -k 10 300 python -u experiments/ab_stream.py --quick > $O/ab_stream_quick.jsonl 2> $O/ab_stream_quick.err && \
timeout -k 10 600 $T tests/test_gpu_int4.py tests/test_gpu_int8.py tests/test_gpu_gemm_tiles.py tests/test_gpu_fuzz.py > $O/pytest_gemm_files.log 2>&1
