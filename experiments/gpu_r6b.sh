set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine_r6b.log 2>&1
timeout -k 10 300 python -u experiments/engine_time.py > gpurun_out/engine_time_r6b.json 2> gpurun_out/engine_time_r6b.err
