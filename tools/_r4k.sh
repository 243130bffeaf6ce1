set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in video-chapter-generation_amd/vcg_hip/libvcg_hip.so video-chapter-generation_amd/build/ab/libvcg_nosum.so video-chapter-generation_amd/build/ab/libvcg_w8.so video-chapter-generation_amd/build/ab/libvcg_w8nosum.so; do
  VCG_LIB_PATH=$lib VCG_RS_DGRAD=1 VCG_BENCH_NOY=1 VCG_BENCH_NOTSM=1 timeout -k 10 120 python tools/bench_dgrad.py "l1" 1 | sed "s#^#$(basename $lib) #" || exit 1
done
