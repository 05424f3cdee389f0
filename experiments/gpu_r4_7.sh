#!/bin/bash
# P = 2 / 4 gloo rehearsals of the multi-GPU bench (8B step + config 5 in both plans), then the
# prefill GEMM counter passes at the routed shapes
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 420 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > $O/r4_rehearsal_p2.jsonl 2> $O/r4_rehearsal_p2.err
rc=$?; echo "p2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --backend gloo --steps 3 --warmup 1 > $O/r4_rehearsal_p4.jsonl 2> $O/r4_rehearsal_p4.err
rc=$?; echo "p4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash experiments/pmc_prefill.sh gpurun_out/r4_pmc_prefill > $O/r4_pmc_prefill.log 2>&1
rc=$?; echo "pmc rc=$rc"
python3 experiments/pmc_prefill_summary.py gpurun_out/r4_pmc_prefill > $O/r4_pmc_prefill.jsonl
exit $rc
