# fp8 actor tests + actor profiles + the full default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_actor_fp8.py > gpurun_out/fp8_tests.log 2>&1 && \
bash scripts/prof_actor.sh && \
timeout -k 10 700 python -u bench.py > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err
