#!/bin/bash
# SQ counters of the genome-gap kernels per configuration (tools/ggap_one.py):
# k_gband score mode, k_gband probability mode, k_ggap probability mode, k_gwin
# probability mode (the default); two
# passes each (8 SQ counters per pass).
# usage (under gpurun): bash tools/pmc_ggap_modes.sh TAG   -> gpurun_out/TAG/<cfg>_pmc{1,2}/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?tag}; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS"
for cfg in "score band" "prob band" "prob rowlane" "prob gwin"; do
  set -- $cfg
  t=$1_$2
  timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $O/${t}_pmc1 -o run -- python3 tools/ggap_one.py $1 $2 200000 3 > $O/${t}_pmc1.out 2> $O/${t}_pmc1.err
  timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $O/${t}_pmc2 -o run -- python3 tools/ggap_one.py $1 $2 200000 3 > $O/${t}_pmc2.out 2> $O/${t}_pmc2.err
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_prob_band -o run -- python3 tools/ggap_one.py prob band 200000 5 > $O/trace_prob_band.out 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_prob_rowlane -o run -- python3 tools/ggap_one.py prob rowlane 200000 5 > $O/trace_prob_rowlane.out 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_prob_gwin -o run -- python3 tools/ggap_one.py prob gwin 200000 5 > $O/trace_prob_gwin.out 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_score_band -o run -- python3 tools/ggap_one.py score band 200000 5 > $O/trace_score_band.out 2>&1
