set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/probe_bw.py
