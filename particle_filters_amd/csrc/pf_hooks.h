// Fault-injection hooks of the GPU tests (tests/test_gpu_resident_launch.py, tests/test_gpu_ledh.py).
// A hook variable (PF_TEST_ABORT, PF_TEST_LEDH_FAIL) takes effect only while PF_TEST_HOOKS=1 is set
// as well, so a stray variable in a production environment cannot change a run.
#pragma once
#include <cstdlib>

#include <hip/hip_runtime.h>

namespace pf {

inline bool test_hook(const char* name) {
  const char* on = std::getenv("PF_TEST_HOOKS");
  if (!(on && std::atoi(on) == 1)) return false;
  const char* e = std::getenv(name);
  return e && std::atoi(e) == 1;
}
// the integer value of a test hook variable (0 unless PF_TEST_HOOKS=1)
inline int test_hook_int(const char* name) {
  const char* on = std::getenv("PF_TEST_HOOKS");
  if (!(on && std::atoi(on) == 1)) return 0;
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : 0;
}

// Uninitialised-LDS regression hook (tests/test_gpu_lds_poison.py): with PF_TEST_LDS_POISON=1 (and
// PF_TEST_HOOKS=1) every launch of the kernels under test is preceded, on its stream, by
// k_lds_poison, which fills the whole 160 KB of LDS of every CU with 0xFFFFFFFF - a NaN as fp32
// and as fp64 - so a kernel that reads an LDS word it did not write sees a NaN, not whatever the
// previous kernel happened to leave (pf_engine.hip).
void lds_poison(hipStream_t s);
void lds_poison_count_add();  // launches made by the hook (pf_test_lds_poison_count)
inline void lds_poison_hook(hipStream_t s) {
  if (test_hook("PF_TEST_LDS_POISON")) {
    lds_poison(s);
    lds_poison_count_add();
  }
}

}  // namespace pf
