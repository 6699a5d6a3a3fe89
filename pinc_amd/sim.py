"""Python handle on one rank of the MI355X PINC simulation (libpinc.so).

This mirrors the reference's run mode regular() (src/main.c:50-304): the
ini file plus ``key=value`` overrides select the operators, normalise the
units and size the population and grids; ``init()`` builds the initial state
and ``step()`` runs one timestep on the GPU.  All computation happens in the
native library; this wrapper only moves arguments and diagnostics.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from . import _lib
from ._lib import HOST, PincSimOpts


class Sim:
    def __init__(self, ini: str, overrides: Sequence[str] = (), *, literal: bool = False,
                 perturb: bool = True, maxwell: bool = False, device_init: bool = False,
                 seed: int = 0, rank: int = 0, nranks: int = 1, device: int = 0,
                 comm_id: bytes | None = None, timing: bool = False, transport=None):
        """transport: a pinc_amd.transport.GlooTransport for multi-rank runs
        without RCCL (several ranks on one GPU, tests); default RCCL."""
        self._id_buf = None
        self._transport = transport
        HOST.pinc_set_host_transport(C.byref(transport.struct) if transport is not None else None)
        opts = PincSimOpts()
        opts.literal = int(literal)
        opts.perturb = int(perturb)
        opts.maxwell = int(maxwell)
        opts.deviceInit = int(device_init)
        opts.seed = seed
        opts.rank = rank
        opts.nranks = nranks
        opts.device = device
        opts.timing = int(timing)
        if comm_id is not None:
            self._id_buf = (C.c_ubyte * len(comm_id)).from_buffer_copy(comm_id)
            opts.commId = C.cast(self._id_buf, C.c_void_p)
        arr = (C.c_char_p * max(1, len(overrides)))(*[o.encode() for o in overrides])
        self._h = HOST.pinc_sim_create(str(ini).encode(), len(overrides), arr, C.byref(opts))
        if not self._h:
            raise RuntimeError("pinc_sim_create failed: " + HOST.pinc_last_error().decode())
        self.nspecies = HOST.pinc_sim_nspecies(self._h)
        self.ndims = HOST.pinc_sim_ndims(self._h)

    # -- lifecycle ---------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            HOST.pinc_sim_free(self._h)
            self._h = None
            if self._transport is not None:
                HOST.pinc_set_host_transport(None)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def init(self) -> None:
        HOST.pinc_sim_init(self._h)

    def step(self, n: int = 1) -> None:
        """n iterations of the main loop (one library call: no return to
        Python between them)."""
        if n == 1:
            HOST.pinc_sim_step(self._h)
        elif n > 1:
            HOST.pinc_sim_steps(self._h, n)

    def op(self, name: str) -> None:
        if HOST.pinc_sim_op(self._h, name.encode()):
            raise ValueError(f"unknown op {name}")

    def sync(self) -> None:
        HOST.pinc_sim_sync(self._h)

    # -- output (the reference's .h5 files) ---------------------------------
    def open_output(self) -> None:
        """pop/rho/phi/E/history files under files:output (main.c:118-131)."""
        HOST.pinc_sim_open_output(self._h)

    def write_output(self, n: float) -> None:
        """main.c:262-266 for step n: E, rho, phi at n, positions at n,
        velocities at n + 0.5, energy rows."""
        HOST.pinc_sim_write_output(self._h, float(n))

    # -- diagnostics -------------------------------------------------------
    def energy(self) -> tuple[float, float, np.ndarray]:
        ke, pe = C.c_double(), C.c_double()
        kes = (C.c_double * self.nspecies)()
        HOST.pinc_sim_energy(self._h, C.byref(ke), C.byref(pe), kes)
        return ke.value, pe.value, np.array(kes)

    @property
    def cycles(self) -> int:
        return HOST.pinc_sim_cycles(self._h)

    def mg_limit(self, max_cycles: int = 0, hist_cap: int = 0) -> None:
        """Cap the V-cycles of one multigrid solve (0: until converged) and
        record up to hist_cap per-cycle RMS residuals (mgSetLimit)."""
        if HOST.pinc_sim_mg_limit(self._h, max_cycles, hist_cap):
            raise RuntimeError("mg_limit: the Poisson solver is not multigrid")

    @property
    def mg_levels(self) -> int:
        """Levels of the multigrid hierarchy in use (0 for the spectral solver)."""
        return HOST.pinc_sim_mg_levels(self._h)

    @property
    def mg_shard(self) -> int:
        """Halo planes of the sharded multigrid level 0 (0: replicated solve)."""
        return HOST.pinc_sim_mg_shard(self._h)

    @property
    def spectral_distributed(self) -> bool:
        """The spectral solve is slab-distributed (no gather of rho)."""
        return bool(HOST.pinc_sim_spectral_distributed(self._h))

    @property
    def obj_collected(self) -> float:
        """Charge the immersed objects collected since init (0 without objects)."""
        return HOST.pinc_sim_obj_collected(self._h)

    def mg_history(self) -> np.ndarray:
        """RMS residual after each V-cycle of the last solve (mgHistory)."""
        n = HOST.pinc_sim_mg_history(self._h, None, 0)
        out = np.zeros(max(n, 0))
        if n > 0:
            HOST.pinc_sim_mg_history(self._h, out.ctypes.data, n)
        return out

    def count(self, s: int) -> int:
        return HOST.pinc_sim_pop_count(self._h, s)

    def total_particles(self) -> int:
        return HOST.pinc_sim_total_particles(self._h)

    def particles(self, s: int) -> tuple[np.ndarray, np.ndarray]:
        n = self.count(s)
        pos = np.zeros((n, self.ndims))
        vel = np.zeros((n, self.ndims))
        HOST.pinc_sim_pop_get(self._h, s, pos.ctypes.data, vel.ctypes.data)
        return pos, vel

    def set_particles(self, s: int, pos: np.ndarray, vel: np.ndarray) -> None:
        pos = np.ascontiguousarray(pos, dtype=np.float64)
        vel = np.ascontiguousarray(vel, dtype=np.float64)
        if HOST.pinc_sim_pop_set(self._h, s, pos.shape[0], pos.ctypes.data, vel.ctypes.data):
            raise RuntimeError("pinc_sim_pop_set failed")

    def grid_shape(self, which: int) -> tuple[int, ...]:
        size = (C.c_int * 4)()
        HOST.pinc_sim_grid_shape(self._h, which, size)
        return tuple(size)

    def grid(self, which: int) -> np.ndarray:
        """rho (0), phi (1) or E (2) in the reference layout (value-major,
        ghost layers included), shaped [nz+2, ny+2, nx+2, nValues] for 3-D."""
        size = self.grid_shape(which)
        rank = self.ndims + 1
        out = np.zeros(int(np.prod(size[:rank])))
        HOST.pinc_sim_grid_get(self._h, which, out.ctypes.data)
        return out.reshape(tuple(reversed(size[:rank])))

    def set_grid(self, which: int, values: np.ndarray) -> None:
        v = np.ascontiguousarray(values, dtype=np.float64).ravel()
        HOST.pinc_sim_grid_set(self._h, which, v.ctypes.data)

    def emigrants(self) -> np.ndarray:
        n = 3 ** self.ndims * self.nspecies
        out = np.zeros(n, dtype=np.int64)
        HOST.pinc_sim_emigrants(self._h, out.ctypes.data)
        return out.reshape(3 ** self.ndims, self.nspecies)

    def species(self) -> tuple[np.ndarray, np.ndarray]:
        q = np.zeros(self.nspecies)
        m = np.zeros(self.nspecies)
        HOST.pinc_sim_species(self._h, q.ctypes.data, m.ctypes.data)
        return q, m

    def timers(self) -> dict[str, float]:
        ms = np.zeros(_lib.NPHASES)
        HOST.pinc_sim_timers(self._h, ms.ctypes.data)
        return dict(zip(_lib.PHASES, ms.tolist()))

    def timers_reset(self) -> None:
        HOST.pinc_sim_timers_reset(self._h)


def h5_available() -> bool:
    return bool(HOST.pinc_h5_available())


def h5_read(path: str, name: str, attr: bool = False) -> np.ndarray:
    """A dataset (or double attribute) of an .h5 file, through the same
    run-time HDF5 binding the writer uses (h5py is not installed)."""
    if attr:
        out = np.zeros(1)
        n = HOST.pinc_h5_read(str(path).encode(), name.encode(), 1, out.ctypes.data, 1)
        if n < 0:
            raise KeyError(f"{path}: attribute {name}")
        return out
    dims = np.zeros(8, dtype=np.int64)
    r = HOST.pinc_h5_dims(str(path).encode(), name.encode(), dims.ctypes.data)
    if r < 0:
        raise KeyError(f"{path}: {name}")
    shape = tuple(int(d) for d in dims[:r])
    out = np.zeros(int(np.prod(shape)) if shape else 1)
    n = HOST.pinc_h5_read(str(path).encode(), name.encode(), 0, out.ctypes.data, out.size)
    if n < 0:
        raise KeyError(f"{path}: {name}")
    return out.reshape(shape)
