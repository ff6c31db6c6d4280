set -o pipefail
mkdir -p gpurun_out
for c in 1 2 4 7; do
  DCA_PIPELINE_CHUNKS=$c timeout -k 10 300 python -u bench.py --actor 0 --steps 10 --warmup 3 > gpurun_out/bench_c$c.log 2>&1 || exit 1
done
