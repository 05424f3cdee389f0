set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine_r6i.log 2>&1
timeout -k 10 300 python -u experiments/engine_time.py > gpurun_out/engine_time_r6i.json 2> gpurun_out/engine_time_r6i.err
timeout -k 10 200 python -u experiments/engine_stamps.py --consumers 7 --dq 1 --ahead 2 --dyn 1 > gpurun_out/engine_stamps7d_r6i.json 2> gpurun_out/engine_stamps_r6i.err
timeout -k 10 200 python -u experiments/engine_stamps.py --consumers 7 --dq 1 --ahead 2 --dyn 0 > gpurun_out/engine_stamps7s_r6i.json 2>> gpurun_out/engine_stamps_r6i.err
timeout -k 10 300 python -u experiments/sweep_gemv.py --graph 14336x4096 > gpurun_out/sweep_14336_r6i.jsonl 2> gpurun_out/sweep_14336_r6i.err
