# round 3, call 20: MALL prefetch of wo's weights riding on the decode attention launch
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_llama_harness.py -m gpu -k "attn or fused" > $O/pytest_attn_pf.log 2>&1 && \
PYTHONPATH=torchao-fork_amd timeout -k 10 300 python -u experiments/probe_mall_gemv.py > $O/probe_mall_gemv.jsonl 2> $O/probe_mall_gemv.err && \
timeout -k 10 900 bash experiments/ab_e2e_args.sh 2 int4wo-32 "--attn_prefetch_wgs 0" "--attn_prefetch_wgs 224" "--attn_prefetch_wgs 96" > $O/ab_e2e_attn_pf.jsonl 2> $O/ab_e2e_attn_pf.err
