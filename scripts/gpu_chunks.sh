# time-chunk pipelining of the exact learner step (recurrence on stream L, heads / weight gradients beside it)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in 1 2 4 8; do
  DCA_PIPELINE_CHUNKS=$c timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --bf16x3-extra 0 --model-5v5-extra 0 --actor 0 --e2e 0 > gpurun_out/chunks_$c.log 2> gpurun_out/chunks_$c.err || exit $?
  echo "chunks=$c $(tail -1 gpurun_out/chunks_$c.log)"
done
