set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gputest.log 2>&1 || { echo "pytest rc=$?" >> gpurun_out/gputest.log; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
TAG=r2i bash tools/profile_round.sh
export CTCEXT_LIB_PATH=$PWD/tools/libctcext_phases.so
timeout -k 10 120 python3 -u tools/diag_phases.py 256 300 128 3 > gpurun_out/ph_cfg3.txt 2>&1 &&
timeout -k 10 120 python3 -u tools/diag_phases.py 128 400 64 1 1000 > gpurun_out/ph_cfg4.txt 2>&1 &&
timeout -k 10 180 python3 -u tools/diag_phases.py 256 100 256 1 5000 > gpurun_out/ph_cfg5.txt 2>&1
