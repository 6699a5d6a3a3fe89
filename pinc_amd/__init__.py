"""pinc_amd -- MI355X-native implementation of PINC's per-timestep PIC hot path.

Native code lives in pinc_amd/lib (built from pinc_amd/csrc and
pinc_amd/host by ``python -m pinc_amd.build``); this package only loads it.
Accessing ``pinc_amd.Sim`` loads the libraries and raises ImportError if they
are missing -- there is no fallback path.  See DESIGN.md.
"""

__all__ = ["Sim"]


def __getattr__(name):
    if name == "Sim":
        from .sim import Sim
        return Sim
    raise AttributeError(name)
