# round 3, call 16: decode attention with whole-line K loads (tao_tune_attn 5): parity, timing, e2e
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_llama_harness.py -m gpu -k attn > $O/pytest_attn5.log 2>&1 && \
timeout -k 10 200 python -u experiments/attn_time.py --modes 0,5 --keys 128,328,512,900 > $O/attn_time5.jsonl 2> $O/attn_time5.err && \
timeout -k 10 700 bash experiments/ab_e2e_args.sh 2 int4wo-32 "--attn_mode 0" "--attn_mode 5" > $O/ab_e2e_attn5.jsonl 2> $O/ab_e2e_attn5.err
