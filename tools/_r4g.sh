set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in video-chapter-generation_amd/vcg_hip/libvcg_hip.so video-chapter-generation_amd/build/ab/libvcg_pf2.so video-chapter-generation_amd/build/ab/libvcg_nt.so video-chapter-generation_amd/build/ab/libvcg_pf2nt.so; do
  echo "== $lib"
  VCG_LIB_PATH=$lib timeout -k 10 200 python tools/bench_bnres.py || exit 1
done
