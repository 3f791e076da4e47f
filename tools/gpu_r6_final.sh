set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/${TAG:-r6z}; mkdir -p $O; cd $R
echo "[$(date +%T)] profile_round" >> $O/steps.log
TAG=${TAG:-r6z} bash tools/profile_round.sh || exit 20
echo "[$(date +%T)] pmc_large_c" >> $O/steps.log
TAG=${TAG:-r6z} bash tools/pmc_large_c.sh || exit 21
echo "[$(date +%T)] done" >> $O/steps.log
