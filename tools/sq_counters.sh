# The decode kernel's instruction mix and wait cycles from SQ counters: two
# rocprofv3 --pmc passes (8 SQ counters each, no tracing beside them) over one
# bench step, then tools/sq_summary.py.  usage (on the box):
#   TAG=r6u CFG=cfg3 bash tools/sq_counters.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/${TAG:-r6u}; mkdir -p $O
export TMPDIR=/tmp
CFG=${CFG:-cfg3}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
B="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT"
n=0
for P in "$A" "$B"; do
  n=$((n + 1))
  echo "[$(date +%T)] pass $n" >> $O/steps.log
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $P -d $O/sq_${CFG}_$n -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu --no-host-io --no-strong > $O/sq_${CFG}_$n.log 2>&1) || exit 30
done
python3 $R/tools/sq_summary.py $O/sq_${CFG}_1/run_counter_collection.csv $O/sq_${CFG}_2/run_counter_collection.csv > $O/sq_${CFG}.txt || exit 31
if [ -n "$SQ_KERNEL2" ]; then SQ_KERNEL=$SQ_KERNEL2 python3 $R/tools/sq_summary.py $O/sq_${CFG}_1/run_counter_collection.csv $O/sq_${CFG}_2/run_counter_collection.csv > $O/sq_${CFG}_k2.txt || exit 32; fi
echo "[$(date +%T)] done" >> $O/steps.log
