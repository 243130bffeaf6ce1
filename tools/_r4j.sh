set -o pipefail
cd $GRAFT_REPO_ROOT
for f in 1 0; do VCG_RS_DGRAD=$f VCG_BENCH_NOY=1 VCG_BENCH_NOTSM=1 timeout -k 10 120 python tools/bench_dgrad.py "l" 1 | sed "s/^/NOTSM RS_DGRAD=$f /" || exit 1; done
