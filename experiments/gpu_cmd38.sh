# round 3, call 28: prefill residual adds fused with the next RMSNorm (tests, e2e A/B)
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_llama_harness.py tests/test_gpu_configs.py -m gpu > $O/pytest_add_norm.log 2>&1 && \
timeout -k 10 700 bash experiments/ab_e2e_args.sh 2 int4wo-32 "--prefill_add_norm 0" "--prefill_add_norm 1" > $O/ab_e2e_add_norm.jsonl 2> $O/ab_e2e_add_norm.err
