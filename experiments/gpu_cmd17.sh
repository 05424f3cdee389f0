# round 3, call 9: stream GEMM timing-only variants (where its time goes), decode attention timing
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 bash experiments/stream_debug.sh run > $O/stream_debug.jsonl 2> $O/stream_debug.err && \
timeout -k 10 200 python -u experiments/attn_time.py --modes 0,4 --keys 128,328,512,900 > $O/attn_time.jsonl 2> $O/attn_time.err
