# round 3, call 26: harness and config-4 oracle tests with the native prefill attention as default
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_llama_harness.py tests/test_gpu_configs.py tests/test_gpu_decode_fused.py tests/test_gpu_decode_fused_int8.py -m gpu > $O/pytest_prefill_default.log 2>&1
