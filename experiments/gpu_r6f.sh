set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine_r6f.log 2>&1
timeout -k 10 200 python -u experiments/engine_stamps.py --consumers 7 > gpurun_out/engine_stamps7_r6f.json 2> gpurun_out/engine_stamps_r6f.err
timeout -k 10 200 python -u experiments/engine_stamps.py --consumers 3 > gpurun_out/engine_stamps3_r6f.json 2>> gpurun_out/engine_stamps_r6f.err
timeout -k 10 300 python -u experiments/engine_time.py > gpurun_out/engine_time_r6f.json 2> gpurun_out/engine_time_r6f.err
