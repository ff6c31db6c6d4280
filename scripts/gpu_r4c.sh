# fp8 encoder forms (numerics + A/B), actor profiles, 5v5 step profile, node-loop actor-precision A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DCA_FP8_ENC_PER_UNIT=0 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_actor_fp8.py > gpurun_out/fp8_tests.log 2>&1 && \
timeout -k 10 120 python -u scripts/enc_fp8_ab.py > gpurun_out/enc_ab.log 2>&1 && \
DCA_FP8_ENC_PER_UNIT=0 bash scripts/prof_actor.sh && \
bash scripts/prof_5v5.sh && \
timeout -k 10 400 python -u scripts/e2e_ab.py 15 2048,12,bf16 2048,12,fp8 2048,14,fp8 > gpurun_out/e2e_ab.log 2> gpurun_out/e2e_ab.err
