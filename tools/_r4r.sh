set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 1 2 1 2; do VCG_WGRAD_PATCH=$v timeout -k 10 120 python tools/bench_wgrad3x3.py || exit 1; done
