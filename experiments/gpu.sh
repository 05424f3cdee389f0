#!/bin/bash
# One GPU-box runner for every measurement recipe (run under gpurun from the repo root):
#   bash experiments/gpu.sh RECIPE TAG [ARGS...]
# Each step runs under its own time limit and the steps are chained: the first failure (a test, a
# fault, a time limit) ends the call. Outputs land in gpurun_out/ (copy what is judged into
# profiles/). Recipes:
#   tests TAG [pytest -k expr]   GPU tests (one process, per-test timeout)
#   bench TAG [bench.py args]    one bench.py line (default: the driver's default run)
#   prof TAG                     rocprofv3 kernel trace + stats of the GEMV-only bench, and the
#                                FETCH_SIZE pass (separate run); digests per shape and per step
#   round_end TAG                tests + smoke + bench + prof (experiments/round_end.sh)
#   pmc_prefill TAG              counter passes of the M = 128 prefill GEMMs (pmc_prefill.sh)
#   py TAG SCRIPT [args]         python experiments/SCRIPT args > gpurun_out/TAG.jsonl
#   rehearse TAG P               bench.py --gpus P --backend gloo on this one GPU (all ranks on it)
#   ab TAG LIB_B SCRIPT [args]   same-box A/B: SCRIPT with the in-tree library, then with LIB_B
#                                (TORCHAO_MI355X_LIB), alternated twice -> gpurun_out/TAG.jsonl
# Several recipes in one call: separate them with "--", e.g.
#   bash experiments/gpu.sh tests r5a -- bench r5a
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp PYTHONPATH=torchao-fork_amd${PYTHONPATH:+:$PYTHONPATH}
O=gpurun_out
mkdir -p $O

run_one() {
  local recipe=$1 tag=$2
  shift 2
  case $recipe in
    tests)
      local k=()
      [ $# -gt 0 ] && k=(-k "$*")
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
        --timeout-method thread -p no:cacheprovider "${k[@]}" > $O/pytest_gpu_$tag.log 2>&1
      local rc=$?; tail -3 $O/pytest_gpu_$tag.log; return $rc ;;
    bench)
      timeout -k 10 600 python -u bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err
      local rc=$?; head -c 600 $O/bench_$tag.json; echo; return $rc ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag \
        -o bench -- python3 bench.py --no-cpu-baseline --no-reference-gpu --no-e2e --no-extras \
        --no-config5 > $O/bench_prof_$tag.json 2> $O/bench_prof_$tag.err || return $?
      timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$tag -o pmc \
        -- python3 bench.py --no-graph --steps 2 --warmup 1 --no-cpu-baseline --no-reference-gpu \
        --no-prefill --no-e2e --no-extras --no-config5 > $O/bench_pmc_$tag.json \
        2> $O/bench_pmc_$tag.err || return $?
      python3 experiments/trace_summary.py "$(find $O/prof_$tag -name "*kernel_trace.csv" | head -1)" \
        129 > $O/trace_summary_$tag.txt
      python3 experiments/pmc_summary.py "$(find $O/pmc_$tag -name "*counter_collection.csv" | head -1)" \
        $O/pmc_fetch_bench_$tag.json 129 ;;
    round_end)
      bash experiments/round_end.sh "$tag" ;;
    pmc_prefill)
      bash experiments/pmc_prefill.sh $O/pmc_prefill_$tag ;;
    py)
      local script=$1
      shift
      timeout -k 10 900 python -u experiments/$script "$@" > $O/$tag.jsonl 2> $O/$tag.err
      local rc=$?; tail -c 1500 $O/$tag.jsonl; return $rc ;;
    ab)
      local lib=$1 script=$2
      shift 2
      for rep in 1 2; do
        echo "{\"ab\": \"A\", \"rep\": $rep}" >> $O/$tag.jsonl
        timeout -k 10 600 python -u experiments/$script "$@" >> $O/$tag.jsonl 2>> $O/$tag.err || return $?
        echo "{\"ab\": \"B\", \"rep\": $rep, \"lib\": \"$lib\"}" >> $O/$tag.jsonl
        TORCHAO_MI355X_LIB=$lib timeout -k 10 600 python -u experiments/$script "$@" \
          >> $O/$tag.jsonl 2>> $O/$tag.err || return $?
      done
      tail -c 1500 $O/$tag.jsonl ;;
    rehearse)  # rehearse TAG P: bench.py's P-rank path on this one GPU (gloo, all ranks on card 0)
      local P=$1
      timeout -k 10 1100 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$P" \
        --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus "$P" --backend gloo \
        --steps 3 --warmup 1 > $O/rehearsal_$tag.jsonl 2> $O/rehearsal_$tag.err
      local rc=$?; grep '^{' $O/rehearsal_$tag.jsonl | head -c 800; echo; return $rc ;;
    *)
      echo "unknown recipe $recipe" >&2; return 2 ;;
  esac
}

args=()
for a in "$@" --; do
  if [ "$a" = "--" ]; then
    if [ ${#args[@]} -gt 0 ]; then
      echo "== ${args[*]}"
      run_one "${args[@]}" || { rc=$?; echo "step '${args[*]}' failed rc=$rc"; exit $rc; }
    fi
    args=()
  else
    args+=("$a")
  fi
done
echo "all steps ok"
