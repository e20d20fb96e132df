set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for m in 1 0; do GRT_SCHEDULE=$m timeout -k 10 120 python3 tools/prof_target.py c3 || exit 1; done
bash tools/gpu_round.sh r01b
