// Error reporting, device discovery and the host DescriptorDistance of liborbgpu.so.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {
thread_local std::string g_last_error;
}

int orbgpu_fail(int code, const char* msg) {
    g_last_error = msg ? msg : "";
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_last_error += " (";
        g_last_error += hipGetErrorString(e);
        g_last_error += ")";
    }
    return code;
}

extern "C" {

const char* orb_last_error(void) { return g_last_error.c_str(); }

int orb_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

// ORBmatcher::DescriptorDistance, reference src/ORBmatcher.cc:2384-2404: popcount(a ^ b) over the
// 8 little-endian 32-bit words of two 256-bit descriptors.
int orb_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    if (!a || !b) return orbgpu_fail(ORB_ERR_ARG, "null descriptor");
    int d = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

}  // extern "C"
