# full default bench after the actor host-loop changes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_vec_actor.py > gpurun_out/vec_tests2.log 2>&1 && \
timeout -k 10 800 python -u bench.py > gpurun_out/bench_r4e.log 2> gpurun_out/bench_r4e.err
