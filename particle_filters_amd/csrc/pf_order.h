// Process-wide order of grid-synchronising launches per device (k_resident, k_ledh_fused).
//
// Their workgroups wait for each other inside the launch, so the grid must be resident at once.
// Two such grids issued on different streams (two handles) could each hold part of the CUs
// and wait for their missing workgroups forever.  A launch on another stream than the previous
// one therefore waits, on the device, for that one to finish (hipStreamWaitEvent: no host sync).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>

namespace pf {

struct GridOrder {
  std::mutex mu;
  hipEvent_t ev[64] = {};
  hipStream_t last[64] = {};
};
inline GridOrder& grid_order() {
  static GridOrder o;  // one per process (inline function: shared by every translation unit)
  return o;
}
inline bool grid_order_off() {  // PF_NO_ORDER=1: diagnostics only (unsafe with several handles)
  static const bool off = [] {
    const char* e = std::getenv("PF_NO_ORDER");
    return e && e[0] == '1';
  }();
  return off;
}
inline void grid_order_begin(int dev, hipStream_t s) {
  if (dev < 0 || dev >= 64 || grid_order_off()) return;
  GridOrder& o = grid_order();
  std::lock_guard<std::mutex> lk(o.mu);
  if (o.ev[dev] && o.last[dev] && o.last[dev] != s) (void)hipStreamWaitEvent(s, o.ev[dev], 0);
}
inline void grid_order_end(int dev, hipStream_t s) {
  if (dev < 0 || dev >= 64 || grid_order_off()) return;
  GridOrder& o = grid_order();
  std::lock_guard<std::mutex> lk(o.mu);
  if (!o.ev[dev] && hipEventCreateWithFlags(&o.ev[dev], hipEventDisableTiming) != hipSuccess) {
    o.ev[dev] = nullptr;
    return;
  }
  if (hipEventRecord(o.ev[dev], s) == hipSuccess) o.last[dev] = s;
}
// a stream about to be destroyed is no longer "the last one" (the event stays valid)
inline void grid_order_forget(int dev, hipStream_t s) {
  if (dev < 0 || dev >= 64) return;
  GridOrder& o = grid_order();
  std::lock_guard<std::mutex> lk(o.mu);
  if (o.last[dev] == s) o.last[dev] = nullptr;
}

}  // namespace pf
