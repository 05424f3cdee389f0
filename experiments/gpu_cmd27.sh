# round 3, call 19: GEMV with MALL-resident vs HBM weights (is a weight prefetch during attention worth it?)
export TMPDIR=/tmp
O=gpurun_out
PYTHONPATH=torchao-fork_amd timeout -k 10 300 python -u experiments/probe_mall_gemv.py > $O/probe_mall_gemv.jsonl 2> $O/probe_mall_gemv.err
