# round 3, call 29: final evidence from the final code, then Llama-3-70B int4wo-32 e2e on one GPU
export TMPDIR=/tmp
O=gpurun_out
bash experiments/round_end.sh r3f && \
(cd torchao-fork_amd && timeout -k 10 900 python3 -u -m torchao._models.llama.generate --model_name Llama-3-70B -q int4wo-32 --num_samples 2 > ../$O/e2e_70b_r3.txt 2> ../$O/e2e_70b_r3.err)
