#!/bin/bash
# scratch GPU command: full GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/full.log 2>&1; echo "pytest rc=$?" >> gpurun_out/full.log
