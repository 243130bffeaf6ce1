// Library-level C ABI: error reporting, version, device handle.
#include "common.h"

#include <vector>

namespace vcg {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// Live per-launch timing of the GEMM kernels (bench.py's dominant-kernel roofline): HIP events
// recorded on the launch stream around each launch while enabled; reduced on query.
struct TimingRec {
  int id;
  hipEvent_t a, b;
  double flops;
};
static std::vector<TimingRec> g_timing;
static bool g_timing_on = false;

int timing_begin(hipStream_t s) {
  if (!g_timing_on) return -1;
  TimingRec r{};
  if (hipEventCreate(&r.a) != hipSuccess || hipEventCreate(&r.b) != hipSuccess) return -1;
  hipEventRecord(r.a, s);
  g_timing.push_back(r);
  return (int)g_timing.size() - 1;
}
void timing_end(int idx, hipStream_t s, int id, double flops) {
  if (idx < 0) return;
  g_timing[idx].id = id;
  g_timing[idx].flops = flops;
  hipEventRecord(g_timing[idx].b, s);
}
static void timing_clear() {
  for (auto& r : g_timing) {
    hipEventDestroy(r.a);
    hipEventDestroy(r.b);
  }
  g_timing.clear();
}
}  // namespace vcg

VCG_API int vcg_timing_enable(int on) {
  vcg::timing_clear();
  vcg::g_timing_on = on != 0;
  return VCG_OK;
}

VCG_API int vcg_timing_query(int kernel_id, double* ms_total, long long* launches, double* flops) {
  double ms = 0.0, fl = 0.0;
  long long n = 0;
  for (auto& r : vcg::g_timing) {
    if (r.id != kernel_id) continue;
    VCG_CHECK_HIP(hipEventSynchronize(r.b));
    float t = 0.f;
    VCG_CHECK_HIP(hipEventElapsedTime(&t, r.a, r.b));
    ms += t;
    fl += r.flops;
    ++n;
  }
  *ms_total = ms;
  *launches = n;
  *flops = fl;
  return VCG_OK;
}

VCG_API const char* vcg_last_error(void) { return vcg::g_last_error.c_str(); }

VCG_API int vcg_version(void) { return 1; }

// Per-device handle: selects the device for the calling thread and checks it is gfx950.
VCG_API int vcg_init(int device) {
  VCG_CHECK_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  VCG_CHECK_HIP(hipGetDeviceProperties(&prop, device));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
    vcg::set_error(std::string("vcg_init: device is ") + prop.gcnArchName + ", libvcg_hip is built for gfx950");
    return VCG_ERR_UNSUPPORTED;
  }
  return VCG_OK;
}

VCG_API int vcg_finalize(void) { return VCG_OK; }

VCG_API int vcg_sync(hipStream_t stream) {
  VCG_CHECK_HIP(hipStreamSynchronize(stream));
  return VCG_OK;
}
