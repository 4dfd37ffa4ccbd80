#!/bin/bash
# SQ counters of k_fill on the headline batch (C3), two passes.
# usage (under gpurun): bash tools/pmc_kfill.sh TAG   -> gpurun_out/TAG/kf{1,2}/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?tag}; mkdir -p $O
B="--steps 3 --warmup 1 --no-cpu --no-side --no-steady"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/kf1 -o run -- python3 bench.py $B > /dev/null 2> $O/kf1.err
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --output-format csv -d $O/kf2 -o run -- python3 bench.py $B > /dev/null 2> $O/kf2.err
