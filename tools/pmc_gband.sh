#!/bin/bash
# SQ counters of the genome-gap kernels on the C4 batch (tools/ggap_ab.py), two passes.
# usage (under gpurun): bash tools/pmc_gband.sh TAG   -> gpurun_out/TAG/pmc{1,2}/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?tag}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc1 -o run -- python3 tools/ggap_ab.py 200000 > $O/pmc1.out 2> $O/pmc1.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --output-format csv -d $O/pmc2 -o run -- python3 tools/ggap_ab.py 200000 > $O/pmc2.out 2> $O/pmc2.err
