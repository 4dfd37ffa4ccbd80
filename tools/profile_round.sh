#!/bin/bash
# Round GPU evidence (run under gpurun): parity tests, the bench line, the
# rocprofv3 kernel-trace summary and the two PMC passes of tools/pmc_traffic.py,
# all on the headline workload (C3).
# usage: bash tools/profile_round.sh TAG [pytest-args]   -> gpurun_out/TAG/...
# back here: tools/keep_profiles.sh TAG  (copies the summaries to profiles/TAG_*)
set -e
TAG=${1:?tag}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $O/pytest_gpu.txt 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
B="--steps 20 --warmup 2 --no-cpu --no-side --no-steady"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $B > $O/trace_bench.json 2> $O/trace.err
B="--steps 3 --warmup 1 --no-cpu --no-side --no-steady"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py $B > /dev/null 2> $O/pmc1.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py $B > /dev/null 2> $O/pmc2.err
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write k_fill $O/traffic.json C3
# genome-gap kernels per mode (k_gband score / probability, k_ggap probability): SQ counters and rocprof summaries
bash tools/pmc_ggap_modes.sh $TAG/ggap_modes
python3 tools/pmc_summary.py $O/ggap_modes/*_pmc1 $O/ggap_modes/*_pmc2 > $O/pmc_ggap_modes.json
