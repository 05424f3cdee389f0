export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_int4.py -x -v --timeout 300 --timeout-method thread -k "aten_identity or aten_convert" > $O/pytest_aten_dequant.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench_r3a.jsonl 2> $O/bench_r3a.err && \
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > $O/rehearsal_p2.jsonl 2> $O/rehearsal_p2.err && \
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --backend gloo --steps 3 --warmup 1 > $O/rehearsal_p4.jsonl 2> $O/rehearsal_p4.err
