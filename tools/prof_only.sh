#!/bin/bash
# rocprofv3 evidence without the test suite (under gpurun): the kernel-trace
# summary of the headline bench, the two traffic PMC passes and k_fill's SQ
# counters (tools/pmc_kfill.sh).
# usage: bash tools/prof_only.sh TAG   -> gpurun_out/TAG/...
set -e
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
B="--steps 20 --warmup 2 --no-cpu --no-side --no-steady"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $B > $O/trace_bench.json 2> $O/trace.err
B="--steps 3 --warmup 1 --no-cpu --no-side --no-steady"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py $B > /dev/null 2> $O/pmc1.err
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py $B > /dev/null 2> $O/pmc2.err
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write k_fill $O/traffic.json C3
bash tools/pmc_kfill.sh $TAG
