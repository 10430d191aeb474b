"""The engine's host code under AddressSanitizer + UndefinedBehaviorSanitizer.

`make -C particle_filters_amd/csrc asan` builds the engine with host-only instrumentation
(`-Xarch_host -fsanitize=address,undefined`; device code is not instrumented) into the C-ABI driver
tests/host/pf_api_asan.cpp.  On the CPU the driver exercises the argument checks and error paths of
include/pf_engine.h; on a GPU it also runs filters (fp32 / fp64, 1-4 replicates, nx 1 and 4), the
device-resident loop, moments, a checkpoint / restore round trip that must continue bitwise, and
the standalone resampler.  Any sanitizer report aborts the driver with a non-zero status.
"""

import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "build", "pf_api_asan")
# leak checking off: the HIP runtime keeps process-lifetime allocations; every other check stays on
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _run(timeout):
    return subprocess.run([EXE], env=ENV, capture_output=True, text=True, timeout=timeout)


def test_host_asan_error_paths_cpu():
    if not os.path.exists(EXE):  # built by __graft_entry__.build(); here if the test runs first
        subprocess.run(["make", "-C", os.path.join(REPO, "particle_filters_amd", "csrc"), "-j8", "asan"],
                       check=True, capture_output=True, timeout=1200)
    r = _run(120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr


@pytest.mark.gpu
def test_host_asan_filter_runs_gpu():
    assert os.path.exists(EXE), "build/pf_api_asan missing: run __graft_entry__.build() (make asan) first"
    r = _run(300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "devices: 0" not in r.stdout, r.stdout
    assert r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
