# round 3, call 25: native prefill attention (tao_attn_prefill_bf16) vs torch's masked SDPA
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_llama_harness.py tests/test_gpu_configs.py -m gpu > $O/pytest_prefill_attn.log 2>&1 && \
PYTHONPATH=torchao-fork_amd timeout -k 10 400 python -u experiments/prefill_profile.py --native > $O/prefill_profile2.jsonl 2> $O/prefill_profile2.err && \
timeout -k 10 700 bash experiments/ab_e2e_args.sh 2 int4wo-32 "--sdpa_prefill" "--native_prefill_attn" > $O/ab_e2e_prefill_attn.jsonl 2> $O/ab_e2e_prefill_attn.err
