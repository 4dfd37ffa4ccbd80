#!/bin/bash
# Round-end GPU evidence (run under gpurun): parity tests, the bench line, the
# rocprofv3 kernel-trace summary and the two PMC passes of tools/pmc_traffic.py.
# usage: bash tools/profile_round.sh TAG      -> profiles/TAG_*
set -e
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-c4 --no-c5 --no-extra > $O/trace_bench.json 2> $O/trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-c4 --no-c5 --no-extra > /dev/null 2> $O/pmc1.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-c4 --no-c5 --no-extra > /dev/null 2> $O/pmc2.err
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write k_fill $O/traffic.json
# back here: cp gpurun_out/TAG/{trace/run_kernel_stats.csv,trace/run_domain_stats.csv,traffic.json,bench.json} profiles/TAG_*
