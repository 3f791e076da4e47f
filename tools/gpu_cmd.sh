#!/bin/bash
# scratch GPU command: parity, then A/B of builds and the phase split
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_properties.py > gpurun_out/par.log 2>&1 || { echo "pytest rc=$?" >> gpurun_out/par.log; exit 1; }
CFG=cfg5 EXTRA="--seq-len 100 --no-host-io" timeout -k 10 300 bash tools/abn.sh 2 abv/ts.so abv/x2.so > gpurun_out/ab.txt 2>&1 || exit 1
CFG=cfg4 EXTRA="--seq-len 400 --no-host-io" timeout -k 10 300 bash tools/abn.sh 2 abv/ts.so abv/x2.so >> gpurun_out/ab.txt 2>&1 || exit 1
export CTCEXT_LIB_PATH=$PWD/tools/libctcext_phases.so
timeout -k 10 180 python3 -u tools/diag_phases.py 256 100 256 1 5000 > gpurun_out/ph_cfg5.txt 2>&1
