#!/bin/bash
# scratch GPU command: large-C parity, phases, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/par.log 2>&1 || { echo "pytest rc=$?" >> gpurun_out/par.log; exit 1; }
export CTCEXT_LIB_PATH=$PWD/tools/libctcext_phases.so
timeout -k 10 120 python3 -u tools/diag_phases.py 128 200 64 1 1000 > gpurun_out/ph_cfg4.txt 2>&1 &&
timeout -k 10 180 python3 -u tools/diag_phases.py 64 40 256 1 5000 > gpurun_out/ph_cfg5.txt 2>&1 || exit 1
unset CTCEXT_LIB_PATH
CFG=cfg4 EXTRA="--seq-len 400 --no-host-io" timeout -k 10 300 bash tools/abn.sh 2 abv/cq2.so abv/cq3.so > gpurun_out/ab.txt 2>&1
CFG=cfg5 EXTRA="--seq-len 100 --no-host-io" timeout -k 10 300 bash tools/abn.sh 1 abv/base4.so abv/cq2.so abv/cq3.so >> gpurun_out/ab.txt 2>&1
