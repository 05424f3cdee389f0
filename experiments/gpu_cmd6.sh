export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_int4.py -x -v --timeout 300 --timeout-method thread -k "aten_identity or aten_convert" > $O/pytest_aten_dequant.log 2>&1
