#!/bin/bash
# usage (under gpurun): bash tools/ab_kfill.sh TAG VARIANT   (VARIANT built by tools/build_variant.sh into gpuexp/)
# A/B of k_fill timing on C3: product vs variant, alternating
O=gpurun_out/$1; mkdir -p $O; V=$2
for i in 1 2; do
  ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/prod$i.json 2>$O/prod$i.err || exit 1
  GSNAPDP_LIB=gpuexp/$V/libgsnapdp.so ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/var$i.json 2>$O/var$i.err || exit 1
done
