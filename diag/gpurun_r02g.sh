set -o pipefail
cd $GRAFT_REPO_ROOT
bash profiles/collect_sq.sh r02a q4k64
