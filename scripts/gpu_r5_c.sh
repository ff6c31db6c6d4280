# round 5 (c): timelines of the exact step — default (32-WG teams, one chunk) and half teams × 4 chunks
set -o pipefail
bash scripts/prof_exact.sh r5_exact_default && \
DCA_TEAM_HALF=1 DCA_PIPELINE_CHUNKS=4 bash scripts/prof_exact.sh r5_exact_h1c4 && \
DCA_PIPELINE_CHUNKS=4 bash scripts/prof_exact.sh r5_exact_h0c4
