set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_lstm_kernel.py tests/test_attn_kernels.py -x -v --timeout 120 --timeout-method thread > gpurun_out/trace_chk_pytest.log 2>&1 && \
 timeout -k 10 120 python -u scripts/lstm_trace.py > gpurun_out/lstm_trace.jsonl 2>&1 && \
 timeout -k 10 120 python -u scripts/lstm_team_trace.py f32 > gpurun_out/team_trace_fwd.jsonl 2>&1 && \
 timeout -k 10 120 python -u scripts/lstm_team_trace.py f32 bwd > gpurun_out/team_trace_bwd.jsonl 2>&1
