# round-5 evidence: profile_round.sh (GPU suite, bench line, rocprof summary, PMC traffic, genome-gap SQ counters)
# plus k_fill's SQ counters; usage: bash tools/r5_final.sh TAG
set -e
TAG=${1:?tag}
bash tools/profile_round.sh $TAG
bash tools/pmc_kfill.sh $TAG
