# round 3, call 7: run length of the per-wave LDS-DMA W stream
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 ./experiments/build/probe_stream5 > $O/probe_stream5.jsonl 2>&1
