"""MI355X-native SIR particle-filter engine.

Drop-in for the SIR inner loop of liyiyang-amber/Particle_filters
(``models/particle_filter.py``): the same ``ParticleFilter`` / ``PFState`` API
over hand-written HIP kernels for gfx950 behind a C ABI (``include/pf_engine.h``,
``libpf_hip.so``), plus the restated ``simulator_*`` data generators.
"""

from . import models, simulators
from .particle_filter import ParticleFilter, PFState, resample_indices

__all__ = ["ParticleFilter", "PFState", "resample_indices", "models", "simulators", "batch"]
__version__ = "0.1.0"
