#!/bin/bash
# GPU-box recipes (run under gpurun from the repo root), one parametrised script instead of
# per-experiment one-offs.  Every GPU step has its own time limit; the chain stops at the
# first failure (set -e), and nothing is retried.
#
#   tools/gpu_round.sh <out-dir> <step> [<step> ...]
#
# steps:
#   tests        the full -m gpu suite (+ smoke)                      -> pytest_gpu.txt, smoke.txt
#   tests:<expr> the -m gpu tests matching -k <expr> (commas for spaces) -> pytest_<expr>.txt
#   bench        python bench.py (the driver's default line)           -> bench_default.json
#   bench:<name>:<args...>   bench.py with args (commas for spaces)     -> bench_<name>.json
#   prof:<name>:<args...>    rocprofv3 --kernel-trace --stats of it     -> prof_<name>/, prof_<name>.json
#   pmc:<name>:<counters>:<args...>  one --pmc pass (counters comma-separated) -> pmc_<name>/
#   trace:<name>:<args...>   rocprofv3 --hip-trace --kernel-trace --stats of it (host API calls) -> trace_<name>/
#   dist:<n>:<args...>       torchrun with n ranks on this box (--allow-wrap) -> dist<n>.json
# e.g. tools/gpu_round.sh gpurun_out/r04 tests bench prof:c5s8:--workload,c5,--steps,5,--no-cpu
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
shift
case "$O" in /*) ;; *) O=$R/$O ;; esac
mkdir -p "$O"
export TMPDIR=/tmp
sp() { echo "$1" | tr ',' ' '; }
for step in "$@"; do
  cd "$R"
  case "$step" in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > "$O/pytest_gpu.txt" 2>&1
      timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > "$O/smoke.txt" 2>&1 ;;
    tests:*)
      k=$(sp "${step#tests:}")
      timeout -k 10 500 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread -k "$k" \
        > "$O/pytest_$(echo "$k" | tr -c 'a-zA-Z0-9_\n' '_').txt" 2>&1 ;;
    bench)
      timeout -k 10 400 python -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" ;;
    bench:*)
      IFS=: read -r _ name args <<< "$step"
      timeout -k 10 400 python -u bench.py $(sp "$args") > "$O/bench_$name.json" 2> "$O/bench_$name.err" ;;
    prof:*)
      IFS=: read -r _ name args <<< "$step"
      cd /tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o prof \
        -- python3 "$R/bench.py" $(sp "$args") > "$O/prof_$name.json" 2> "$O/prof_$name.err" ;;
    trace:*)
      IFS=: read -r _ name args <<< "$step"
      cd /tmp
      timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$O/trace_$name" -o trace \
        -- python3 "$R/bench.py" $(sp "$args") > "$O/trace_$name.json" 2> "$O/trace_$name.err" ;;
    pmc:*)
      IFS=: read -r _ name ctrs args <<< "$step"
      cd /tmp
      timeout -s KILL 240 rocprofv3 --pmc $(sp "$ctrs") -d "$O/pmc_$name" -o pmc --output-format csv \
        -- python3 "$R/bench.py" --no-cpu --settle-ms 0 $(sp "$args") > /dev/null 2> "$O/pmc_$name.err" ;;
    dist:*)
      IFS=: read -r _ n args <<< "$step"
      timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
        --master-port $((29500 + n)) bench.py --gpus "$n" --allow-wrap $(sp "$args") > "$O/dist$n.json" 2> "$O/dist$n.err" ;;
    *)
      echo "gpu_round.sh: unknown step $step" >&2; exit 2 ;;
  esac
done
