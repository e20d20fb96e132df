set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for v in pre cur pre cur; do GRT_LIB=variants/$v/libgrt.so GRT_LIB_ALLOW_MISSING=1 timeout -k 10 300 python3 tools/c4_shard_time.py 8 0 | sed "s/^/$v /" || exit 1; done
