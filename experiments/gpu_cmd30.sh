# round 3, call 21: decode attention with 32 keys per wave step (one round trip up to 512 keys)
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_llama_harness.py -m gpu -k attn > $O/pytest_attn6.log 2>&1 && \
timeout -k 10 200 python -u experiments/attn_time.py --modes 0,6 --keys 128,200,328,512,900 > $O/attn_time6.jsonl 2> $O/attn_time6.err && \
timeout -k 10 700 bash experiments/ab_e2e_args.sh 2 int4wo-32 "--attn_mode 0" "--attn_mode 6" > $O/ab_e2e_attn6.jsonl 2> $O/ab_e2e_attn6.err
