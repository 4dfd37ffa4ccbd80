#!/bin/bash
# k_gwin diagnostics under gpurun: the GW_PROF build's per-phase cycles, then the
# A/B against k_ggap (tools/gwin_ab.py).  usage: bash tools/gwin_round.sh TAG [n]
O=gpurun_out/$1; mkdir -p $O; N=${2:-50000}
GSNAPDP_LIB=gmap-gsnap_amd/lib_prof/libgsnapdp.so timeout -k 10 300 python -u tools/gwin_prof.py $N 200000 > $O/prof.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/gwin_ab.py $N $O/gwin_ab.json > $O/ab.txt 2>&1
