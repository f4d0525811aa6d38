set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/ab_bitwise.sh base sel
