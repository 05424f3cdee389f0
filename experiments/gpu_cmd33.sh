# round 3, call 24: where the config-4 prefill spends its time
export TMPDIR=/tmp
O=gpurun_out
PYTHONPATH=torchao-fork_amd timeout -k 10 400 python -u experiments/prefill_profile.py > $O/prefill_profile.jsonl 2> $O/prefill_profile.err
