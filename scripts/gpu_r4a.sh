# exact-step profile (fast activations) + PMC of the exact kernels + the full default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/prof_exact.sh profx2 && bash scripts/pmc_exact.sh && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r4a.log 2> gpurun_out/bench_r4a.err
