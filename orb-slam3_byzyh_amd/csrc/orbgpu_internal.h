// Internal helpers shared by the liborbgpu.so translation units (not part of the C ABI).
#pragma once

// Record `msg` as this thread's last error (orb_last_error) and return `code`.
int orbgpu_fail(int code, const char* msg);
