# round 3, call 10: fused-decode row blocks per workgroup (per-op sweep, e2e A/B with the
# attention kernel choice)
export TMPDIR=/tmp
O=gpurun_out
PYTHONPATH=torchao-fork_amd timeout -k 10 300 python -u experiments/bench_decode.py --bpw 1,2,3,4,7,8 > $O/bench_decode_bpw.jsonl 2> $O/bench_decode_bpw.err && \
timeout -k 10 900 bash experiments/ab_e2e_args.sh 2 int4wo-32 "" "--decode_bpw 4" "--attn_mode 4" "--decode_bpw 4 --attn_mode 4" > $O/ab_e2e_bpw_attn.jsonl 2> $O/ab_e2e_bpw_attn.err
