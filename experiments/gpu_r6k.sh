set -e
mkdir -p gpurun_out
B=experiments/ablib/libnibold.so
for rep in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-reference-gpu --no-e2e --no-extras --no-config5 --no-prefill > gpurun_out/ab_nib_A${rep}_r6k.json 2>> gpurun_out/ab_nib_r6k.err
  TORCHAO_MI355X_LIB=$B timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-reference-gpu --no-e2e --no-extras --no-config5 --no-prefill > gpurun_out/ab_nib_B${rep}_r6k.json 2>> gpurun_out/ab_nib_r6k.err
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_int4.py tests/test_gpu_decode_fused.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_nib_r6k.log 2>&1
