# round 3, call 27: Llama-3-70B int4wo-32 e2e on one GPU with the current harness
export TMPDIR=/tmp
O=gpurun_out
(cd torchao-fork_amd && timeout -k 10 900 python3 -u -m torchao._models.llama.generate --model_name Llama-3-70B -q int4wo-32 --num_samples 2 > ../$O/e2e_70b_r3.txt 2> ../$O/e2e_70b_r3.err)
