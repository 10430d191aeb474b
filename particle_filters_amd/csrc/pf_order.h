// Process-wide order of grid-synchronising launches per device (k_resident, k_ledh_fused).
//
// Their workgroups wait for each other inside the launch, so the grid must be resident at once.
// Two such grids issued on different streams (two handles) could each hold part of the CUs
// and wait for their missing workgroups forever.  A launch on another stream than the previous
// one therefore waits, on the device, for that one to finish (hipStreamWaitEvent: no host sync).
// The event is recorded lazily: only when a grid comes on another stream, on the previous stream
// at that moment (it then covers everything issued there so far, that grid included - a wait
// that can only be longer than needed, never shorter).  Runs that stay on one stream queue no
// marker at all (one marker packet cost ~5 us of wall time per resident run, profiles/r04/ab).
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
// Scope of one or more grid-synchronising launches on stream s: the process-wide lock is held
// from before the wait on the previous grid's event until this grid's event is recorded, so two
// host threads driving different handles cannot both pass the wait before either records
// (their grids would then be issued unordered).  Construct right before the launches; the
// event is recorded by end() or, on an early return, by the destructor.
class GridOrderScope {
 public:
  GridOrderScope(int dev, hipStream_t s) : dev_(dev), s_(s) {
    if (dev < 0 || dev >= 64 || grid_order_off()) return;
    lk_ = std::unique_lock<std::mutex>(grid_order().mu);
    GridOrder& o = grid_order();
    if (o.last[dev] && o.last[dev] != s) {
      if (!o.ev[dev] && hipEventCreateWithFlags(&o.ev[dev], hipEventDisableTiming) != hipSuccess) o.ev[dev] = nullptr;
      // no event: nothing to order by but the host (rare: event creation failed)
      if (!o.ev[dev] || hipEventRecord(o.ev[dev], o.last[dev]) != hipSuccess || hipStreamWaitEvent(s, o.ev[dev], 0) != hipSuccess)
        (void)hipStreamSynchronize(o.last[dev]);
    }
  }
  void end() {
    if (!lk_.owns_lock()) return;
    grid_order().last[dev_] = s_;
    lk_.unlock();
  }
  ~GridOrderScope() { end(); }
  GridOrderScope(const GridOrderScope&) = delete;
  GridOrderScope& operator=(const GridOrderScope&) = delete;

 private:
  int dev_;
  hipStream_t s_;
  std::unique_lock<std::mutex> lk_;
};
// a stream about to be destroyed is no longer "the last one" (the event stays valid)
inline void grid_order_forget(int dev, hipStream_t s) {
  if (dev < 0 || dev >= 64) return;
  GridOrder& o = grid_order();
  std::lock_guard<std::mutex> lk(o.mu);
  if (o.last[dev] == s) o.last[dev] = nullptr;
}

}  // namespace pf
