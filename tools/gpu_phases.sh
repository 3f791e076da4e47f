#!/bin/bash
# per-phase cycle split (diagnostics build tools/libctcext_phases.so) for cfg3, cfg4 and cfg5 shapes
set -o pipefail
mkdir -p gpurun_out
export CTCEXT_LIB_PATH=${PHASES_LIB:-$PWD/tools/libctcext_phases.so}
timeout -k 10 120 python3 -u tools/diag_phases.py 256 300 128 3 > gpurun_out/ph_cfg3.txt 2>&1 &&
timeout -k 10 120 python3 -u tools/diag_phases.py 128 400 64 1 1000 > gpurun_out/ph_cfg4.txt 2>&1 &&
timeout -k 10 180 python3 -u tools/diag_phases.py 256 100 256 1 5000 > gpurun_out/ph_cfg5.txt 2>&1
