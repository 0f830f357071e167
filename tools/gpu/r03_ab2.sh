set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=ab_upd bash tools/gpu/ab_lib.sh && TAG=c3ab bash tools/gpu/c3_ab.sh
