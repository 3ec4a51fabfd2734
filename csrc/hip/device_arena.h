// Per-device state kept across sweep calls: grow-only device buffers, one stream, two timing
// events and the CU count.
//
// A tuning session calls the sweep kernels many times with similar sizes (one call per trace,
// per objective, per shard of `tune --distributed`). Allocating, creating events and querying
// device properties on every call cost more than a small sweep's kernel (hipMalloc/hipFree of the
// output buffers alone run to milliseconds); here they happen once per device and size class.
// Calls on one device serialize on the arena's mutex -- they would share the GPU anyway -- and
// the arenas live for the process: freeing them from a static destructor could run after the HIP
// runtime has shut down.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>

namespace ksa_gpu {

struct DeviceArena {
  std::mutex mu;
  int dev = -1;
  int cus = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  static constexpr int kSlots = 8;
  void* buf[kSlots] = {};
  size_t cap[kSlots] = {};

  // Device buffer `slot` with room for at least `bytes` (contents undefined). Grows by at least
  // 1.5x so that a sequence of slightly larger requests does not reallocate every time.
  hipError_t get(int slot, size_t bytes, void** out) {
    if (slot < 0 || slot >= kSlots) return hipErrorInvalidValue;
    if (bytes == 0) bytes = 1;
    if (cap[slot] < bytes) {
      if (buf[slot]) {
        // the stream may still read the old buffer (a failed call returns early)
        (void)hipStreamSynchronize(stream);
        (void)hipFree(buf[slot]);
        buf[slot] = nullptr;
        cap[slot] = 0;
      }
      const size_t want = bytes + bytes / 2;
      const hipError_t e = hipMalloc(&buf[slot], want);
      if (e != hipSuccess) {
        buf[slot] = nullptr;
        return e;
      }
      cap[slot] = want;
    }
    *out = buf[slot];
    return hipSuccess;
  }
};

// Synchronizes the stream when the call's frame unwinds, so that no early error return leaves a
// copy in flight from a host buffer that is about to be freed, or into the caller's output.
struct StreamDrain {
  hipStream_t stream;
  ~StreamDrain() { (void)hipStreamSynchronize(stream); }
};

// The arena of device `dev`, created (stream, events, CU count) on first use. On failure returns
// nullptr and sets *err.
inline DeviceArena* device_arena(int dev, std::string* err) {
  static std::mutex map_mu;
  static std::map<int, std::unique_ptr<DeviceArena>>* arenas = new std::map<int, std::unique_ptr<DeviceArena>>();
  std::lock_guard<std::mutex> lock(map_mu);
  auto it = arenas->find(dev);
  if (it != arenas->end()) return it->second.get();
  std::unique_ptr<DeviceArena> a(new DeviceArena());
  a->dev = dev;
  hipError_t e = hipSetDevice(dev);
  hipDeviceProp_t prop;
  if (e == hipSuccess) e = hipGetDeviceProperties(&prop, dev);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&a->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&a->e0);
  if (e == hipSuccess) e = hipEventCreate(&a->e1);
  if (e != hipSuccess) {
    *err = std::string("device arena: ") + hipGetErrorString(e);
    if (a->e0) (void)hipEventDestroy(a->e0);
    if (a->e1) (void)hipEventDestroy(a->e1);
    if (a->stream) (void)hipStreamDestroy(a->stream);
    return nullptr;
  }
  a->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  DeviceArena* raw = a.get();
  (*arenas)[dev] = std::move(a);
  return raw;
}

}  // namespace ksa_gpu
