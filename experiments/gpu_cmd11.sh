# round 3, call 3: streaming skeleton of an unsplit prefill tile (intake floor), decode attention timing
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 ./experiments/build/probe_stream > $O/probe_stream.jsonl 2>&1 && \
timeout -k 10 200 python -u experiments/attn_time.py --modes 0,4 --keys 128,200,328,512 > $O/attn_time.jsonl 2> $O/attn_time.err
