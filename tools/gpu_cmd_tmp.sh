set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -m pytest tests/test_trajectory.py -m gpu -q -rA -p no:cacheprovider > gpurun_out/traj.log 2>&1
echo "pytest rc=$?"
