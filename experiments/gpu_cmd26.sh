# round 3, call 18: stream GEMM with K phases rotated per workgroup (cold shared weight tiles)
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_gemm_stream.py > $O/pytest_stream_rot.log 2>&1 && \
timeout -k 10 400 python -u experiments/ab_stream.py --quick > $O/ab_stream_rot.jsonl 2> $O/ab_stream_rot.err
