set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --actor 0 --e2e 0 --e2e-5v5-extra 0 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 && \
 cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py gpurun_out/prof/run_results.db --steps 9 > gpurun_out/prof_summary.md && rm -rf gpurun_out/prof && \
 timeout -k 10 120 python -u scripts/lstm_team_trace.py f32 > gpurun_out/team_trace_fwd.jsonl 2>&1 && \
 timeout -k 10 120 python -u scripts/lstm_team_trace.py f32 bwd > gpurun_out/team_trace_bwd.jsonl 2>&1
