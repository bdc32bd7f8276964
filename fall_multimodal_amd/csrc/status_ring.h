// Host side of a device error word: a kernel that can fail on the device (a group barrier that timed
// out) raises an int flag in device memory; after every launch that can raise it, post() enqueues a
// copy of the flag into the next slot of a ring of pinned host words (one event each), so a flag is
// never overwritten by a later call's copy before the host has read it. take() folds the completed
// copies into `sticky` and reports a raised flag once as F3_EDEVICE. Used by TARGCN (GRU group
// barriers) and the 3-stream net (the sensor branch's cooperative CNN1D).
#pragma once
#include <hip/hip_runtime.h>

#include "common.h"

#ifndef F3_EDEVICE
#define F3_EDEVICE 1005
#endif

namespace f3 {

inline bool stream_capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess) {
    (void)hipGetLastError();
    return true;
  }
  return cs != hipStreamCaptureStatusNone;
}

struct StatusRing {
  static constexpr int R = 16;
  int* host = nullptr;  // [R] pinned
  hipEvent_t ev[R] = {};
  int head = 0, count = 0;  // oldest pending slot, number of pending copies
  bool sticky = false;

  StatusRing() = default;
  StatusRing(const StatusRing&) = delete;
  StatusRing& operator=(const StatusRing&) = delete;
  // Called from the owner's destroy entry point (f3_*_destroy), while the HIP runtime is alive; the
  // owners are never static objects, so nothing here runs from exit-time destructors.
  ~StatusRing() {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (host) (void)hipHostFree(host);
  }

  void fold(int i) {
    sticky = sticky || host[i] != 0;
    host[i] = 0;
    head = (i + 1) % R;
    --count;
  }

  // fold the completed copies (oldest first; wait: all of them); a flag raised by any earlier call
  // -> F3_EDEVICE once (then cleared)
  int take(bool wait) {
    while (count > 0) {
      const int i = head;
      if (wait) {
        if (hipEventSynchronize(ev[i]) != hipSuccess) return F3_EHIP;
      } else if (hipEventQuery(ev[i]) != hipSuccess) {
        (void)hipGetLastError();
        break;  // later copies are behind this one in stream order
      }
      fold(i);
    }
    if (!sticky) return F3_OK;
    sticky = false;
    return F3_EDEVICE;
  }

  // enqueue the copy of the device word `flag` on stream s (a full ring first waits for its oldest
  // copy). Under stream capture nothing is enqueued: a replayed graph has no host to report to.
  int post(const int* flag, hipStream_t s) {
    if (stream_capturing(s)) return F3_OK;
    if (!host) {
      if (hipHostMalloc(&host, sizeof(int) * R, hipHostMallocDefault) != hipSuccess) {
        host = nullptr;
        return F3_EHIP;
      }
      for (int i = 0; i < R; ++i) host[i] = 0;
    }
    if (count == R) {
      if (hipEventSynchronize(ev[head]) != hipSuccess) return F3_EHIP;
      fold(head);
    }
    const int slot = (head + count) % R;
    if (!ev[slot] && hipEventCreateWithFlags(&ev[slot], hipEventDisableTiming) != hipSuccess) return F3_EHIP;
    if (hipMemcpyAsync(host + slot, flag, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess) return F3_EHIP;
    if (hipEventRecord(ev[slot], s) != hipSuccess) return F3_EHIP;
    ++count;
    return F3_OK;
  }
};

}  // namespace f3
