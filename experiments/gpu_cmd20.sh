# round 3, call 12: intake by load pattern (half-line MFMA-order loads vs full lines)
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 ./experiments/build/probe_l2_pattern > $O/probe_l2_pattern.jsonl 2>&1
