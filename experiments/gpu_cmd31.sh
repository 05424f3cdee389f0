# round 3, call 22: k decode steps per HIP graph launch (parity, e2e A/B)
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_llama_harness.py -m gpu -k "graph_decode" > $O/pytest_multistep.log 2>&1 && \
timeout -k 10 900 bash experiments/ab_e2e_args.sh 2 int4wo-32 "--steps_per_graph 1" "--steps_per_graph 8" "--steps_per_graph 32" > $O/ab_e2e_multistep.jsonl 2> $O/ab_e2e_multistep.err
