# round 3, call 5: run-length sweep of the per-step ring skeleton
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 ./experiments/build/probe_stream3 > $O/probe_stream3.jsonl 2>&1
