set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine_r6g.log 2>&1
timeout -k 10 200 python -u experiments/engine_stamps.py --consumers 7 --dq 1 > gpurun_out/engine_stamps7_r6g.json 2> gpurun_out/engine_stamps_r6g.err
timeout -k 10 200 python -u experiments/engine_stamps.py --consumers 3 --dq 1 > gpurun_out/engine_stamps3_r6g.json 2>> gpurun_out/engine_stamps_r6g.err
timeout -k 10 300 python -u experiments/engine_time.py > gpurun_out/engine_time_r6g.json 2> gpurun_out/engine_time_r6g.err
