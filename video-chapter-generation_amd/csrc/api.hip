// Library-level C ABI: error reporting, version, device handle.
#include "common.h"

#include <cstdio>
#include <map>
#include <mutex>
#include <vector>

namespace vcg {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// Live per-launch timing of the GEMM kernels (bench.py's dominant-kernel roofline): HIP events
// recorded on the launch stream around each launch while enabled; reduced on query.
struct TimingRec {
  int id;
  hipEvent_t a, b;
  double flops, bytes;  // algorithmic work of the launch (bytes: every operand read once, outputs written once)
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
void timing_end(int idx, hipStream_t s, int id, double flops, double bytes) {
  if (idx < 0) return;
  g_timing[idx].id = id;
  g_timing[idx].flops = flops;
  g_timing[idx].bytes = bytes;
  hipEventRecord(g_timing[idx].b, s);
}
static void timing_clear() {
  for (auto& r : g_timing) {
    hipEventDestroy(r.a);
    hipEventDestroy(r.b);
  }
  g_timing.clear();
}

// GEMM census: which kernel ran which GEMM shape (tests and bench.py compare the benchmarked step with the
// oracle-anchored one); the host dispatches from one thread, the mutex keeps it safe anyway
static std::mutex g_census_mu;
static std::map<std::string, long long> g_census;
static bool g_census_on = false;
bool census_on() { return g_census_on; }
void census_add(const char* tag, long long M, long long N, long long K) {
  if (!g_census_on) return;
  char key[192];
  snprintf(key, sizeof(key), "%s M=%lld N=%lld K=%lld", tag, M, N, K);
  std::lock_guard<std::mutex> lock(g_census_mu);
  ++g_census[key];
}
}  // namespace vcg

VCG_API int vcg_gemm_census_enable(int on) {
  std::lock_guard<std::mutex> lock(vcg::g_census_mu);
  vcg::g_census.clear();
  vcg::g_census_on = on != 0;
  return VCG_OK;
}

VCG_API int vcg_gemm_census_size(void) {
  std::lock_guard<std::mutex> lock(vcg::g_census_mu);
  return (int)vcg::g_census.size();
}

VCG_API int vcg_gemm_census_get(int i, char* key, int n, long long* count) {
  std::lock_guard<std::mutex> lock(vcg::g_census_mu);
  VCG_REQUIRE(i >= 0 && i < (int)vcg::g_census.size() && key && n > 0 && count, "bad census index / buffer");
  auto it = vcg::g_census.begin();
  std::advance(it, i);
  snprintf(key, (size_t)n, "%s", it->first.c_str());
  *count = it->second;
  return VCG_OK;
}

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

// Per-launch roofline: ideal = max(flops / peak_flops, bytes / peak_bytes_per_s) of each launch, summed.
VCG_API int vcg_timing_roofline(int kernel_id, double peak_tflops, double peak_gbs, double* ms_total,
                                double* ideal_ms, double* bytes, double* flops) {
  VCG_REQUIRE(peak_tflops > 0.0 && peak_gbs > 0.0, "peaks must be positive");
  double ms = 0.0, ideal = 0.0, by = 0.0, fl = 0.0;
  for (auto& r : vcg::g_timing) {
    if (r.id != kernel_id) continue;
    VCG_CHECK_HIP(hipEventSynchronize(r.b));
    float t = 0.f;
    VCG_CHECK_HIP(hipEventElapsedTime(&t, r.a, r.b));
    ms += t;
    const double tf = r.flops / (peak_tflops * 1e12), tb = r.bytes / (peak_gbs * 1e9);
    ideal += 1e3 * (tf > tb ? tf : tb);
    by += r.bytes;
    fl += r.flops;
  }
  *ms_total = ms;
  *ideal_ms = ideal;
  *bytes = by;
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
