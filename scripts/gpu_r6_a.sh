# round 6 (a): GPU suite + smoke after the vendor-GEMM cleanup (bf16 learner branch / attn.hip removed), then the
# headline bench with the node loop at the default 2 s hand-off deadline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6a_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6a_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err
echo "exit $?"
