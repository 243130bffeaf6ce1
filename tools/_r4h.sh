set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r4h VCG_RS1X1 0 1 2
