#!/bin/bash
# same-box kernel profiles of the bench step with and without BN-on-load (bn2 -> conv3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VCG_BNIN=1 bash tools/r02_prof.sh bnon && bash tools/r02_prof.sh bnoff
