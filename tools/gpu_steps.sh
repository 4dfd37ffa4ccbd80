#!/bin/bash
# One parameterised GPU launcher (run under gpurun): each named step writes under
# gpurun_out/TAG/, runs under its own time limit, and the first failing step ends
# the call (no GPU step runs after a failure).
#   bash tools/gpu_steps.sh TAG STEP [STEP ...]
# steps:
#   tests      pytest -m gpu (parity suite)                       -> pytest_gpu.txt
#   pc267      tools/pc_check.py gpu on gpudata/pc267.npz          -> pc267.json
#   bench      bench.py (full default run, CPU legs included)      -> bench.json
#   quick      bench.py --steps 20 --warmup 3 --no-cpu             -> bench.json
#   trace      rocprofv3 --kernel-trace --stats of the C3 bench    -> trace/
#   traffic    FETCH_SIZE / WRITE_SIZE passes + tools/pmc_traffic.py -> traffic.json
#   kfill_sq   k_fill SQ counters (tools/pmc_kfill.sh)             -> kf1/ kf2/
#   ggap_modes genome-gap SQ counters per mode                     -> ggap_modes/, pmc_ggap_modes.json
#   slices     the N = 2/4/8 slices' per-rank steps (tools/slice_trace.py 8)
set -o pipefail
TAG=${1:?tag}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
B3="--steps 3 --warmup 1 --no-cpu --no-side --no-steady"
for s in "$@"; do
  echo "[$(date +%T)] step $s"
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
             > $O/pytest_gpu.txt 2>&1; rc=$?; tail -1 $O/pytest_gpu.txt ;;
    pc267) timeout -k 10 300 python -u tools/pc_check.py gpu gpudata/pc267.npz $O/pc267.json > $O/pc267.txt 2>&1
           rc=$?; tail -3 $O/pc267.txt ;;
    bench) timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; rc=$? ;;
    quick) timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > $O/bench.json 2> $O/bench.err; rc=$? ;;
    trace) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
             python3 bench.py --steps 20 --warmup 2 --no-cpu --no-side --no-steady > $O/trace_bench.json \
             2> $O/trace.err; rc=$? ;;
    traffic) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
               python3 bench.py $B3 > /dev/null 2> $O/pmc1.err &&
             timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
               python3 bench.py $B3 > /dev/null 2> $O/pmc2.err &&
             python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write k_fill $O/traffic.json C3; rc=$? ;;
    kfill_sq) bash tools/pmc_kfill.sh $TAG; rc=$? ;;
    ggap_modes) bash tools/pmc_ggap_modes.sh $TAG/ggap_modes &&
                python3 tools/pmc_summary.py $O/ggap_modes/*_pmc1 $O/ggap_modes/*_pmc2 > $O/pmc_ggap_modes.json
                rc=$? ;;
    slices) timeout -k 10 300 python tools/slice_trace.py 8 0 30 > $O/slices.txt 2>&1; rc=$? ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "step $s failed rc=$rc"
    exit $rc
  fi
done
echo "[$(date +%T)] all steps ok"
