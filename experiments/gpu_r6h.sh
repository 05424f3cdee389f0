set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine_r6h.log 2>&1
timeout -k 10 300 python -u experiments/engine_time.py > gpurun_out/engine_time_r6h.json 2> gpurun_out/engine_time_r6h.err
timeout -k 10 200 python -u experiments/engine_stamps.py --consumers 7 --dq 1 --ahead 3 > gpurun_out/engine_stamps7_r6h.json 2> gpurun_out/engine_stamps_r6h.err
timeout -k 10 300 python -u experiments/sweep_gemv.py --graph 14336x4096 > gpurun_out/sweep_14336_r6h.jsonl 2> gpurun_out/sweep_14336_r6h.err
