"""pinc_amd -- MI355X-native implementation of PINC's per-timestep PIC hot path.

Native code lives in pinc_amd/lib (built from pinc_amd/csrc and
pinc_amd/host); this package only loads it.  See DESIGN.md.
"""
from .sim import Sim  # noqa: F401  (raises ImportError if the native libs are missing)

__all__ = ["Sim"]
