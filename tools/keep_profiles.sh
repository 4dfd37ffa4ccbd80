#!/bin/bash
# Copy one profile_round.sh run's summaries into profiles/ (tracked).
# usage: tools/keep_profiles.sh TAG
set -e
TAG=${1:?tag}
O=gpurun_out/$TAG
cp $O/trace/run_kernel_stats.csv profiles/${TAG}_c3_kernel_stats.csv
cp $O/trace/run_domain_stats.csv profiles/${TAG}_c3_domain_stats.csv 2>/dev/null || true
cp $O/traffic.json profiles/${TAG}_traffic.json
cp $O/bench.json profiles/${TAG}_bench.json
cp $O/pytest_gpu.txt profiles/${TAG}_pytest_gpu.txt
cp $O/pmc_ggap_modes.json profiles/${TAG}_pmc_ggap_modes.json 2>/dev/null || true
