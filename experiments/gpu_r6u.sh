#!/bin/bash
# round-6 evidence on the final library: full GPU suite, smoke, FETCH passes + bench line +
# kernel trace (evidence.sh), prefill counter passes
set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r6u.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6u.log 2>&1
bash experiments/evidence.sh r6u
bash experiments/pmc_prefill.sh gpurun_out/pmc_prefill_r6u
