# round 3, call 13: k-split tiles 32x64 / 64x32 / 128x16 (W read by one workgroup), parity + A/B
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_gemm_ksplit.py > $O/pytest_ksplit.log 2>&1 && \
timeout -k 10 400 python -u experiments/ab_ksplit.py --quick --rot > $O/ab_ksplit_rot.jsonl 2> $O/ab_ksplit_rot.err
