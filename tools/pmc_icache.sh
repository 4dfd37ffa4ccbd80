#!/bin/bash
# Instruction-fetch counters of k_fill on the headline batch (C3): the SQ pass of
# pmc_kfill.sh plus the instruction-cache pass, each a run of its own.
# usage (under gpurun): bash tools/pmc_icache.sh TAG   -> gpurun_out/TAG/{kf2,ic}/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?tag}; mkdir -p $O
B="--steps 3 --warmup 1 --no-cpu --no-side --no-steady"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/kf2 -o run -- python3 bench.py $B > /dev/null 2> $O/kf2.err
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_REQ --output-format csv -d $O/ic -o run -- python3 bench.py $B > /dev/null 2> $O/ic.err
