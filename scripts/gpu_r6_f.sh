# round 6 (f): GPU featurization — its GPU tests + the actor / ingest tests it touches, the full bench (raw-staged actor
# runtime and node loop, pipelined policy-step rates), actor kernel summaries (copies on SDMA, featurize kernel)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_featurize.py \
  tests/test_vec_actor.py tests/test_actor_gpu.py tests/test_offpolicy.py tests/test_packing.py \
  > gpurun_out/r6f_gpu_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/r6f_bench.json 2> gpurun_out/r6f_bench.err || exit $?
for P in fp32 bf16 fp8; do
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profa_$P -o run -- python3 $R/scripts/actor_bench.py 2048 $P > $R/gpurun_out/profa_$P.log 2>&1 || exit $?
  cd $R && python scripts/prof_summary.py gpurun_out/profa_$P/run_results.db --steps 213 > gpurun_out/r6_actor_${P}_summary.md && rm -rf gpurun_out/profa_$P || exit $?
done
echo done
