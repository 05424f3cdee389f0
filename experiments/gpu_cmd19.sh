# round 3, call 11: k-split prefill GEMM parity tests and A/B; decode tests after the attention /
# head routing change
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_gemm_ksplit.py > $O/pytest_ksplit.log 2>&1 && \
timeout -k 10 400 python -u experiments/ab_ksplit.py --quick > $O/ab_ksplit_quick.jsonl 2> $O/ab_ksplit_quick.err && \
timeout -k 10 400 $T tests/test_llama_harness.py tests/test_gpu_decode_fused.py -m gpu > $O/pytest_decode.log 2>&1 && \
# weight loads at the default cache policy (libkdef.so) instead of non-temporal
TORCHAO_MI355X_LIB=experiments/build/libkdef.so timeout -k 10 400 python -u experiments/ab_ksplit.py --quick > $O/ab_ksplit_quick_wdef.jsonl 2> $O/ab_ksplit_quick_wdef.err
