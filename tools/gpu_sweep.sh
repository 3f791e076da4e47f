set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/parity_sweep.py 400 > gpurun_out/sweep.txt 2>&1
