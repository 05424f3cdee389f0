# round 3, call 15: decode prologue loads kept ahead of the weight loads (no vmcnt(0) before the
# first slices): fused-decode tests, per-op timing new vs previous library, e2e A/B
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_decode_fused.py tests/test_gpu_decode_fused_int8.py > $O/pytest_prologue.log 2>&1 && \
PYTHONPATH=torchao-fork_amd timeout -k 10 300 python -u experiments/bench_decode.py > $O/bench_decode_new.jsonl 2> $O/bench_decode_new.err && \
PYTHONPATH=torchao-fork_amd TORCHAO_MI355X_LIB=experiments/build/libprev.so timeout -k 10 300 python -u experiments/bench_decode.py > $O/bench_decode_prev.jsonl 2> $O/bench_decode_prev.err && \
timeout -k 10 700 bash experiments/ab_e2e.sh /root/repo/experiments/build/libprev.so int4wo-32 2 > $O/ab_e2e_prologue.txt 2> $O/ab_e2e_prologue.err && \
timeout -k 10 500 bash experiments/ab_e2e.sh /root/repo/experiments/build/libprev.so int8wo 1 > $O/ab_e2e_prologue_int8wo.txt 2>> $O/ab_e2e_prologue.err && \
timeout -k 10 500 bash experiments/ab_e2e.sh /root/repo/experiments/build/libprev.so int8dq 1 > $O/ab_e2e_prologue_int8dq.txt 2>> $O/ab_e2e_prologue.err
