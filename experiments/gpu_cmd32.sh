# round 3, call 23: final evidence from the final code (tests, smoke, bench, rocprof, FETCH_SIZE),
# then the int8 e2e modes with the current harness defaults
export TMPDIR=/tmp
O=gpurun_out
bash experiments/round_end.sh r3d && \
(cd torchao-fork_amd && for q in int8wo int8dq; do timeout -k 10 300 python3 -m torchao._models.llama.generate -q $q --num_samples 3 2>/dev/null | tail -1; done) > $O/e2e_int8_r3d.jsonl
