#!/bin/bash
# C4 genome-gap stage timing (tools/ablate_ggap.py) for the product and each variant in gpuexp/
# usage (under gpurun): bash tools/ab_ggap.sh TAG MODE(prob|score) VARIANT...
O=gpurun_out/$1; M=$2; shift 2; mkdir -p $O
timeout -k 10 300 python3 tools/ablate_ggap.py $M > $O/prod.txt 2>$O/prod.err || exit 1
for v in "$@"; do
  GSNAPDP_LIB=gpuexp/$v/libgsnapdp.so timeout -k 10 300 python3 tools/ablate_ggap.py $M > $O/$v.txt 2>$O/$v.err || exit 1
done
timeout -k 10 300 python3 tools/ablate_ggap.py $M > $O/prod2.txt 2>$O/prod2.err || exit 1
