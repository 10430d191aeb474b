// Fault-injection hooks of the GPU tests (tests/test_gpu_resident_launch.py, tests/test_gpu_ledh.py).
// A hook variable (PF_TEST_ABORT, PF_TEST_LEDH_FAIL) takes effect only while PF_TEST_HOOKS=1 is set
// as well, so a stray variable in a production environment cannot change a run.
#pragma once
#include <cstdlib>

namespace pf {

inline bool test_hook(const char* name) {
  const char* on = std::getenv("PF_TEST_HOOKS");
  if (!(on && std::atoi(on) == 1)) return false;
  const char* e = std::getenv(name);
  return e && std::atoi(e) == 1;
}

}  // namespace pf
