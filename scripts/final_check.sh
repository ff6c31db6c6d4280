# Round-end record on one MI355X: GPU test suite, smoke, full bench (all extra fields), 1v1 and 5v5 kernel profiles.
# Outputs under gpurun_out/ (copy the summaries into profiles/).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.log 2> gpurun_out/bench_final.err && \
bash scripts/prof_exact.sh profx && bash scripts/prof_1v1.sh && bash scripts/prof_5v5.sh
