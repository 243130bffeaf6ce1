// Library-level C ABI: error reporting, version, device handle.
#include "common.h"

namespace vcg {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace vcg

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
