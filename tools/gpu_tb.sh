set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/${TAG:-tb}; mkdir -p $O; cd $R
export LD_LIBRARY_PATH=$R/ctc-beam-search-op_amd/ctcext_amd/lib
timeout -k 10 60 ./tools/traceback_unit > $O/unit_seg.txt 2>&1; rc=$?; echo "rc=$rc" >> $O/unit_seg.txt; [ $rc -le 1 ] || exit 10
CTCEXT_TRACEBACK=0 timeout -k 10 60 ./tools/traceback_unit > $O/unit_old.txt 2>&1; rc=$?; echo "rc=$rc" >> $O/unit_old.txt; [ $rc -le 1 ] || exit 11
timeout -k 10 120 python tools/diag_traceback.py > $O/diag.txt 2>&1 || exit 12
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "paper or edge or single_class or record_ring or global_state_tier_shapes or full_length_golden or cfg3_full" > $O/focus.log 2>&1 || exit 13
echo done >> $O/unit_seg.txt
