# round 3 (re-entry), call 1: full evidence of the current code, then the P=2 / P=4 gloo rehearsals
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
bash experiments/round_end.sh r3a && \
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > $O/rehearsal_p2.jsonl 2> $O/rehearsal_p2.err && \
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --backend gloo --steps 3 --warmup 1 > $O/rehearsal_p4.jsonl 2> $O/rehearsal_p4.err
