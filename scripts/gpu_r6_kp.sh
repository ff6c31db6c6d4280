# round 6: final GPU suite + smoke (scripts/gpu_r6_k.sh), then the actor launch-shape A/B (scripts/gpu_r6_p.sh)
set -o pipefail
bash scripts/gpu_r6_k.sh || exit $?
bash scripts/gpu_r6_p.sh
