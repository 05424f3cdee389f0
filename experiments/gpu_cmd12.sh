# round 3, call 4: x-resident register-stream skeleton (intake floor without per-step barriers)
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 ./experiments/build/probe_stream2 > $O/probe_stream2.jsonl 2>&1
