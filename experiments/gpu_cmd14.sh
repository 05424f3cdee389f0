# round 3, call 6: W stream by registers vs LDS-DMA, with and without the x tile
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 ./experiments/build/probe_stream4 > $O/probe_stream4.jsonl 2>&1
