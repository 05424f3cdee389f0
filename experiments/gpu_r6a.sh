set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --ignore tests/test_gpu_engine.py > gpurun_out/pytest_gpu_r6a.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6a.log 2>&1
bash experiments/evidence.sh r6a
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine_r6a.log 2>&1
timeout -k 10 300 python -u experiments/engine_time.py > gpurun_out/engine_time_r6a.json 2> gpurun_out/engine_time_r6a.err
