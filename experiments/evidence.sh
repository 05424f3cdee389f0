#!/bin/bash
# One gpurun session's measurement evidence (round 6): the FETCH_SIZE passes, then the default
# bench line that reads them (roofline.traffic, int8wo_m1 traffic), then a rocprofv3 kernel trace
# of the bench whose per-step kernel sum is checked against the lines (step_trace_summary.py).
# Usage: bash experiments/evidence.sh TAG   (outputs in gpurun_out/; copy what is judged to profiles/)
set -e
T=${1:-r6}
O=gpurun_out
export TMPDIR=/tmp
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$T -o pmc -- \
  python3 bench.py --no-graph --steps 2 --warmup 1 --no-cpu-baseline --no-reference-gpu \
  --no-prefill --no-e2e --no-extras --no-config5 > $O/bench_pmc_$T.json 2> $O/bench_pmc_$T.err
python3 experiments/pmc_summary.py "$(find $O/pmc_$T -name "*counter_collection.csv" | head -1)" \
  $O/pmc_fetch_bench_$T.json 129 > /dev/null
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc8_$T -o pmc -- \
  python3 experiments/int8wo_pmc.py run > $O/int8wo_pmc_$T.log 2>&1
python3 experiments/int8wo_pmc.py summarize \
  "$(find $O/pmc8_$T -name "*counter_collection.csv" | head -1)" $O/pmc_fetch_int8wo_$T.json > /dev/null
timeout -k 10 480 python3 -u bench.py --pmc-file $O/pmc_fetch_bench_$T.json \
  --pmc-int8wo-file $O/pmc_fetch_int8wo_$T.json > $O/bench_$T.json 2> $O/bench_$T.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o bench -- \
  python3 bench.py --no-cpu-baseline --no-reference-gpu --no-e2e --no-extras --no-config5 \
  --no-prefill --pmc-file $O/pmc_fetch_bench_$T.json > $O/bench_prof_$T.json 2> $O/bench_prof_$T.err
TR="$(find $O/prof_$T -name "*kernel_trace.csv" | head -1)"
python3 experiments/step_trace_summary.py "$TR" $O/bench_prof_$T.json $O/step_trace_$T.json > /dev/null
python3 experiments/step_trace_summary.py "$TR" $O/bench_$T.json $O/step_trace_vs_default_$T.json > /dev/null
echo done > $O/evidence_$T.ok
