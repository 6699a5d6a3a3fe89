"""ctypes wrapper of the CPU oracle (oracle/build/liborc.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product (pinc_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path
from typing import Sequence

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "liborc.so"


def _load() -> C.CDLL:
    if not LIB_PATH.exists():
        subprocess.run(["make", "-s", "-C", str(HERE), "-j4"], check=True)
    lib = C.CDLL(str(LIB_PATH))
    vp = C.c_void_p
    sigs = {
        "orc_world_new": (vp, [C.c_char_p, C.c_int, C.POINTER(C.c_char_p), C.c_int]),
        "orc_world_free": (None, [vp]),
        "orc_world_init": (None, [vp, C.c_int, C.c_int, C.c_ulonglong]),
        "orc_world_init_fields": (None, [vp]),
        "orc_world_step": (None, [vp]),
        "orc_world_nranks": (C.c_int, [vp]),
        "orc_world_cycles": (C.c_long, [vp]),
        "orc_world_solves": (C.c_long, [vp]),
        "orc_world_energy": (None, [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), vp]),
        "orc_world_species": (None, [vp, vp, vp]),
        "orc_op": (None, [vp, C.c_char_p]),
        "orc_grid_shape": (C.c_long, [vp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]),
        "orc_grid_get": (None, [vp, C.c_int, C.c_int, C.c_int, vp]),
        "orc_grid_set": (None, [vp, C.c_int, C.c_int, C.c_int, vp]),
        "orc_pop_count": (C.c_long, [vp, C.c_int, C.c_int]),
        "orc_pop_get": (None, [vp, C.c_int, C.c_int, vp, vp, vp]),
        "orc_pop_set": (None, [vp, C.c_int, C.c_int, C.c_long, vp, vp, vp]),
        "orc_mpi_emigrants": (None, [vp, C.c_int, vp]),
        "orc_mpi_thresholds": (None, [vp, C.c_int, vp]),
        "orc_mpi_emigrant_buffer": (C.c_long, [vp, C.c_int, C.c_int, vp]),
        "orc_mpi_alloc": (None, [vp, C.c_int, vp]),
        "orc_kat_acc": (None, [C.c_int, vp, C.c_int, vp, C.c_long, vp, vp, C.c_double, C.c_double, C.c_int, vp]),
        "orc_kat_distr": (None, [C.c_int, vp, C.c_int, vp, C.c_long, vp, C.c_double, C.c_int]),
        "orc_kat_neighbor_to_rank": (C.c_int, [vp, vp, C.c_int]),
        "orc_kat_rank_to_neighbor": (C.c_int, [vp, vp, C.c_int]),
        "orc_kat_reciprocal": (C.c_int, [C.c_int, C.c_int]),
        "orc_kat_neighborhood": (None, [C.c_char_p, vp, vp]),
        "orc_kat_extract": (None, [C.c_char_p, C.c_int, vp, vp, vp, vp, C.c_int, vp, vp, C.c_long, vp]),
        "orc_world_ndims": (C.c_int, [vp]),
        "orc_world_mg_limit": (None, [vp, C.c_long, C.c_long]),
        "orc_world_mg_history": (C.c_long, [vp, vp, C.c_long]),
        "orc_set_threads": (None, [C.c_int]),
        "orc_world_mg_levels": (C.c_int, [vp]),
        "orc_world_timers": (None, [vp, vp]),
        "orc_world_nspecies": (C.c_int, [vp]),
        "orc_discrete_poisson": (None, [C.c_int, vp, vp, vp]),
        "oo_create": (vp, [vp, vp]),
        "oo_free": (None, [vp]),
        "oo_capacitance": (None, [vp, vp]),
        "oo_apply": (None, [vp, vp, vp]),
        "oo_collect": (None, [vp, vp]),
        "oo_init_collect": (None, [vp, vp]),
        "oo_step": (None, [vp, vp]),
        "oo_nobjects": (C.c_int, [vp]),
        "oo_nsurface": (C.c_long, [vp, C.c_int]),
        "oo_ninterior": (C.c_long, [vp, C.c_int]),
        "oo_surface_nodes": (None, [vp, C.c_int, vp]),
        "oo_interior_nodes": (None, [vp, C.c_int, vp]),
        "oo_collected": (C.c_double, [vp, C.c_int]),
        "oo_rho_obj": (None, [vp, vp]),
        "oo_set_reference_divisor": (None, [vp, C.c_int]),
    }
    for n, (r, a) in sigs.items():
        f = getattr(lib, n)
        f.restype = r
        f.argtypes = a
    return lib


LIB = _load()


class World:
    """All subdomains of a run, emulated in one process (orc_sim.c)."""

    def __init__(self, ini: str, overrides: Sequence[str] = (), literal: bool = False):
        arr = (C.c_char_p * max(1, len(overrides)))(*[o.encode() for o in overrides])
        self._h = LIB.orc_world_new(str(ini).encode(), len(overrides), arr, int(literal))
        self.nranks = LIB.orc_world_nranks(self._h)

    def close(self):
        if self._h:
            LIB.orc_world_free(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def init(self, perturb=True, maxwell=False, seed=0):
        LIB.orc_world_init(self._h, int(perturb), int(maxwell), seed)

    def init_fields(self):
        LIB.orc_world_init_fields(self._h)

    def step(self, n=1):
        for _ in range(n):
            LIB.orc_world_step(self._h)

    def op(self, name: str):
        LIB.orc_op(self._h, name.encode())

    @property
    def cycles(self):
        return LIB.orc_world_cycles(self._h)

    def mg_limit(self, max_cycles: int = 0, hist_cap: int = 0):
        """Cap the V-cycles of one solve (0: until converged) and record up
        to hist_cap per-cycle RMS residuals."""
        LIB.orc_world_mg_limit(self._h, max_cycles, hist_cap)

    PHASES = ["move", "migrate", "deposit", "solve", "efield", "accelerate", "energy"]

    def timers(self) -> dict:
        """Wall seconds per phase of ow_step since creation."""
        out = np.zeros(7)
        LIB.orc_world_timers(self._h, out.ctypes.data)
        return dict(zip(self.PHASES, out.tolist()))

    def mg_history(self) -> np.ndarray:
        n = LIB.orc_world_mg_history(self._h, None, 0)
        out = np.zeros(n)
        if n:
            LIB.orc_world_mg_history(self._h, out.ctypes.data, n)
        return out

    def energy(self):
        ke, pe = C.c_double(), C.c_double()
        LIB.orc_world_energy(self._h, C.byref(ke), C.byref(pe), None)
        return ke.value, pe.value

    def grid(self, which: int, rank: int = 0, level: int = 0) -> np.ndarray:
        size = (C.c_int * 4)()
        n = LIB.orc_grid_shape(self._h, rank, which, level, size)
        out = np.zeros(n)
        LIB.orc_grid_get(self._h, rank, which, level, out.ctypes.data)
        rank = self.ndims + 1
        # reference layout: value index fastest -> reversed shape
        return out.reshape(tuple(reversed([size[i] for i in range(rank)])))

    def set_grid(self, which: int, values: np.ndarray, rank: int = 0, level: int = 0):
        v = np.ascontiguousarray(values, dtype=np.float64).ravel()
        LIB.orc_grid_set(self._h, rank, which, level, v.ctypes.data)

    def count(self, s: int, rank: int = 0) -> int:
        return LIB.orc_pop_count(self._h, rank, s)

    def particles(self, s: int, rank: int = 0):
        n = self.count(s, rank)
        nd = self.ndims
        pos = np.zeros((n, nd))
        vel = np.zeros((n, nd))
        ids = np.zeros(n, dtype=np.int64)
        LIB.orc_pop_get(self._h, rank, s, pos.ctypes.data, vel.ctypes.data, ids.ctypes.data)
        return pos, vel, ids

    def set_particles(self, s: int, pos, vel, ids=None, rank: int = 0):
        pos = np.ascontiguousarray(pos, dtype=np.float64)
        vel = np.ascontiguousarray(vel, dtype=np.float64)
        idp = None
        if ids is not None:
            ids = np.ascontiguousarray(ids, dtype=np.int64)
            idp = ids.ctypes.data
        LIB.orc_pop_set(self._h, rank, s, pos.shape[0], pos.ctypes.data, vel.ctypes.data, idp)

    def emigrants(self, rank: int = 0) -> np.ndarray:
        n = 3 ** self.ndims * self.nspecies
        out = np.zeros(n, dtype=np.int64)
        LIB.orc_mpi_emigrants(self._h, rank, out.ctypes.data)
        return out.reshape(3 ** self.ndims, self.nspecies)

    def emigrant_records(self, ne: int, rank: int = 0) -> np.ndarray:
        """emigrants[ne] of the last extraction: one row (pos, vel) per record."""
        n = LIB.orc_mpi_emigrant_buffer(self._h, rank, ne, None)
        out = np.zeros((n, 2 * self.ndims))
        if n:
            LIB.orc_mpi_emigrant_buffer(self._h, rank, ne, out.ctypes.data)
        return out

    @property
    def ndims(self) -> int:
        return LIB.orc_world_ndims(self._h)

    @property
    def nspecies(self) -> int:
        return LIB.orc_world_nspecies(self._h)

    def species(self):
        q = np.zeros(self.nspecies)
        m = np.zeros(self.nspecies)
        LIB.orc_world_species(self._h, q.ctypes.data, m.ctypes.data)
        return q, m


def run_steps(ini: str, overrides: Sequence[str], steps: int, literal=False, perturb=True,
              maxwell=False, seed=0):
    """KE/PE history of a run (n = 1..steps) and the V-cycle counts."""
    w = World(ini, overrides, literal)
    w.init(perturb, maxwell, seed)
    w.init_fields()
    ke, pe, cyc = [], [], []
    for _ in range(steps):
        w.step()
        k, p = w.energy()
        ke.append(k)
        pe.append(p)
        cyc.append(w.cycles)
    w.close()
    return np.array(ke), np.array(pe), np.array(cyc)


class Objects:
    """Immersed objects of a one-subdomain World (orc_obj.c, object.c
    restated with its defects corrected).  mask: [z, y, x] object ids over
    the true nodes."""

    def __init__(self, world: "World", mask):
        m = np.ascontiguousarray(mask, dtype=np.float64)
        self.w = world
        self._h = LIB.oo_create(world._h, m.ctypes.data)
        self.n = LIB.oo_nobjects(self._h)

    def close(self):
        if self._h:
            LIB.oo_free(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def surface(self, a: int = 0) -> np.ndarray:
        out = np.zeros(LIB.oo_nsurface(self._h, a), dtype=np.int64)
        LIB.oo_surface_nodes(self._h, a, out.ctypes.data)
        return out

    def interior(self, a: int = 0) -> np.ndarray:
        out = np.zeros(LIB.oo_ninterior(self._h, a), dtype=np.int64)
        LIB.oo_interior_nodes(self._h, a, out.ctypes.data)
        return out

    def capacitance(self):
        LIB.oo_capacitance(self._h, self.w._h)

    def apply(self) -> np.ndarray:
        pc = np.zeros(max(1, self.n))
        LIB.oo_apply(self._h, self.w._h, pc.ctypes.data)
        return pc[:self.n]

    def collect(self):
        LIB.oo_collect(self._h, self.w._h)

    def reference_divisor(self, on: bool = True):
        """Spread collected charge with object.c:476-478's cumulative
        divisor 1/lookupSurfaceOffset[a+1] (the reference's defect)."""
        LIB.oo_set_reference_divisor(self._h, int(on))

    def init_collect(self):
        LIB.oo_init_collect(self._h, self.w._h)

    def step(self, n: int = 1):
        for _ in range(n):
            LIB.oo_step(self.w._h, self._h)

    def collected(self, a: int = 0) -> float:
        return LIB.oo_collected(self._h, a)

    def rho_obj(self) -> np.ndarray:
        g = self.w.grid(0)
        out = np.zeros(g.size)
        LIB.oo_rho_obj(self._h, out.ctypes.data)
        return out.reshape(g.shape)
