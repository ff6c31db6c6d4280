set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_5v5_head.py 1400 > gpurun_out/r5_diag_5v5_head4.txt 2>&1
echo "diag rc=$?"
