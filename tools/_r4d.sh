set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in video-chapter-generation_amd/vcg_hip/libvcg_hip.so video-chapter-generation_amd/build/ab/libvcg_nb6.so; do
  echo "== $lib"
  VCG_LIB_PATH=$lib VCG_BENCH_NOY=1 timeout -k 10 120 python tools/bench_dgrad.py "" 1 || exit 1
done
