set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine_r6j.log 2>&1
timeout -k 10 300 python -u experiments/engine_time.py > gpurun_out/engine_time_r6j.json 2> gpurun_out/engine_time_r6j.err
timeout -k 10 200 python -u experiments/engine_stamps.py > gpurun_out/engine_stamps_r6j.json 2> gpurun_out/engine_stamps_r6j.err
cd torchao-fork_amd
for e in 0 1 0 1; do
  timeout -k 10 240 python -u -m torchao._models.llama.generate -q int4wo-32 --num_samples 3 --ffn_engine $e >> ../gpurun_out/e2e_engine_ab_r6j.jsonl 2>> ../gpurun_out/e2e_engine_ab_r6j.err
done
