// device_scope.hpp -- selects a device for the HIP calls of a scope and restores the calling
// thread's device after it. Every entry point runs on its caller's thread (a cgo call runs on the
// goroutine's OS thread, a Python call on the interpreter's), which may be using another device;
// the library must not leave that thread on a device it did not choose.
#pragma once

#include <hip/hip_runtime.h>

struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int d) {
    if (hipGetDevice(&prev) != hipSuccess) {
      (void)hipGetLastError();
      prev = -1;
    }
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};
