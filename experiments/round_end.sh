#!/bin/bash
# Round-end evidence on one GPU box (run under gpurun): GPU tests, smoke, the default bench line,
# its rocprofv3 kernel trace + stats, and a FETCH_SIZE counter pass (separate run, no tracing
# domains besides the kernel trace). Everything lands in gpurun_out/; copy what is judged into
# profiles/. Usage: bash experiments/round_end.sh TAG
set -e
T=${1:-r1}
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu_$T.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > $O/smoke_$T.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_$T.json 2> $O/bench_$T.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o bench -- \
  python3 bench.py --no-cpu-baseline --no-reference-gpu --no-e2e --no-extras --no-config5 > $O/bench_prof_$T.json \
  2> $O/bench_prof_$T.err
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$T -o pmc -- \
  python3 bench.py --no-graph --steps 2 --warmup 1 --no-cpu-baseline --no-reference-gpu \
  --no-prefill --no-e2e --no-extras --no-config5 > $O/bench_pmc_$T.json 2> $O/bench_pmc_$T.err
# digests (CPU only): per-shape kernel durations of the trace, HBM bytes per shape and step
python3 experiments/trace_summary.py "$(find $O/prof_$T -name "*kernel_trace.csv" | head -1)" 129 \
  > $O/trace_summary_$T.txt
python3 experiments/pmc_summary.py "$(find $O/pmc_$T -name "*counter_collection.csv" | head -1)" \
  $O/pmc_fetch_bench_$T.json 129
echo done > $O/round_end_$T.ok
