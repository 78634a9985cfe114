set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/profile.sh r06m c4 c4 && bash tools/profile.sh r06m prod prod
