# round 3, call 17: RCCL collectives captured in a HIP graph with the HIP linears (1-rank nccl group)
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_rccl_graph.py tests/test_distributed_cpu.py -m gpu > $O/pytest_rccl_graph.log 2>&1
