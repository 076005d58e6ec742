// Host-side resource keying of the forward's C-ABI (ground.hip), written
// against a small device API so that the keying is testable without a GPU
// (tests/test_host.py compiles it with a mock API): a call's pinned header
// buffer, side streams and events belong to the device of the stream (or
// graph) it runs on, not to whatever device the calling thread has current.
//   Api::get_device(int *dev), Api::set_device(int dev),
//   Api::stream_device(void *stream, int *dev) — 0 on success.
#pragma once
#include <map>

namespace rnnl {

// Makes `dev` the current device for the guard's scope (restored after).
template <class Api>
struct DeviceGuardT {
  int prev = -1;
  explicit DeviceGuardT(int dev) {
    int cur = 0;
    if (dev >= 0 && Api::get_device(&cur) == 0 && cur != dev && Api::set_device(dev) == 0) prev = cur;
  }
  ~DeviceGuardT() {
    if (prev >= 0) (void)Api::set_device(prev);
  }
  DeviceGuardT(const DeviceGuardT &) = delete;
  DeviceGuardT &operator=(const DeviceGuardT &) = delete;
};

// The device of a stream argument: a null stream is the current device's.
template <class Api>
int stream_device_of(void *stream) {
  int dev = 0;
  if (stream) return Api::stream_device(stream, &dev) == 0 ? dev : -1;
  return Api::get_device(&dev) == 0 ? dev : -1;
}

// The current device's entry of a per-device map (callers hold a
// DeviceGuardT for the device of their data / stream); nullptr when the
// current device cannot be read.
template <class Api, class Res>
Res *current_device_entry(std::map<int, Res> &all, int *dev_out = nullptr) {
  int dev = 0;
  if (Api::get_device(&dev) != 0) return nullptr;
  if (dev_out) *dev_out = dev;
  return &all[dev];
}

}  // namespace rnnl
