"""CPU oracle for the SIR particle-filter hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``particle_filters_amd/`` may import this
package; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker.

Parity pinned: ``tests/golden/*.npz`` hold outputs of the reference itself
(``/root/reference``, imported in the build container by
``tests/golden/make_golden.py``); ``tests/test_oracle_golden.py`` checks this
oracle reproduces them bit-for-bit (fp64).
"""
