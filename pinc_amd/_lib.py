"""ctypes binding of the native MI355X PINC libraries (pinc_amd/lib).

The product path has no fallback: if libpinc.so / libpinc_hip.so are missing
or fail to load, importing this module raises.  Build with
``python -m pinc_amd.build``.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

# PINC_LIBDIR: an alternative in-tree build (kernel-variant experiments)
LIBDIR = Path(os.environ.get("PINC_LIBDIR") or Path(__file__).resolve().parent / "lib")
PINC_COMM_ID_BYTES = 128
NPHASES = 8
PHASES = ["move", "extract", "migrate", "deposit", "solve", "efield", "accelerate", "energy"]


class PincSimOpts(C.Structure):
    _fields_ = [
        ("literal", C.c_int),
        ("perturb", C.c_int),
        ("maxwell", C.c_int),
        ("deviceInit", C.c_int),
        ("seed", C.c_ulonglong),
        ("rank", C.c_int),
        ("nranks", C.c_int),
        ("device", C.c_int),
        ("commId", C.c_void_p),
        ("timing", C.c_int),
    ]


def _load() -> tuple[C.CDLL, C.CDLL]:
    hip_path = LIBDIR / "libpinc_hip.so"
    host_path = LIBDIR / "libpinc.so"
    if not hip_path.exists() or not host_path.exists():
        raise ImportError(f"native PINC libraries not built ({LIBDIR}); run python -m pinc_amd.build")
    # One ROCm stack per process.  libpinc_hip.so needs libamdhip64.so.7,
    # librocfft.so.0 and librccl.so.1; torch bundles its own copies with the
    # same sonames but links them under unversioned names.  Loaded first, the
    # system (/opt/rocm) copies do not satisfy torch's names, so torch brings
    # a second HIP/HSA runtime into the process: the second one to touch the
    # GPU finds no device (KFD serves one runtime per process), and in round
    # 1 the two copies aborted at exit in their teardown (a double free) --
    # that was the import-order dependence.  Loading torch first makes the
    # loader satisfy our sonames with torch's already-loaded stack, whichever
    # module the caller imported first; a process without torch (the C
    # driver, tests/c_driver) runs on /opt/rocm.  RTLD_LOCAL keeps our
    # symbols out of the global scope; libpinc finds libpinc_hip by rpath.
    # PINC_TORCH_STACK=0 skips the pre-import (a torch-free Python process
    # then runs on /opt/rocm like the C driver; it must not import torch
    # afterwards).  runtime_stack() reports which copies a process mapped.
    if os.environ.get("PINC_TORCH_STACK", "1") != "0":
        try:
            import torch  # noqa: F401  (see above: binds our libraries to torch's ROCm stack)
        except ImportError:
            pass
    hip = C.CDLL(str(hip_path), mode=C.RTLD_LOCAL)
    host = C.CDLL(str(host_path), mode=C.RTLD_LOCAL)
    return hip, host


HIP, HOST = _load()
# this process sets its world through PincSimOpts (rank, size, device, RCCL
# id): the library must not read launcher variables (torchrun's RANK etc.)
HOST.pinc_world_explicit()


def runtime_stack() -> dict:
    """The HIP runtime, rocFFT and RCCL files this process has mapped: torch's
    bundled copies for Python entry points (torch imported first, see _load),
    /opt/rocm for the C driver and PINC_TORCH_STACK=0.  The libraries are
    built against /opt/rocm's headers (ROCm 7.2); torch's bundled runtime is
    its own release (torch.version.hip), used through the stable HIP C ABI."""
    out = {}
    try:
        for line in Path("/proc/self/maps").read_text().splitlines():
            f = line.split()[-1] if line.count("/") else ""
            for key in ("libamdhip64", "librocfft", "librccl"):
                if key in f and key not in out:
                    out[key] = f
    except OSError:
        pass
    return out

_sigs = {
    "pinc_last_error": (C.c_char_p, []),
    "pinc_sim_create": (C.c_void_p, [C.c_char_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(PincSimOpts)]),
    "pinc_sim_free": (None, [C.c_void_p]),
    "pinc_sim_init": (C.c_int, [C.c_void_p]),
    "pinc_sim_step": (C.c_int, [C.c_void_p]),
    "pinc_sim_steps": (C.c_int, [C.c_void_p, C.c_int]),
    "pinc_sim_op": (C.c_int, [C.c_void_p, C.c_char_p]),
    "pinc_sim_energy": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "pinc_sim_cycles": (C.c_long, [C.c_void_p]),
    "pinc_sim_mg_limit": (C.c_int, [C.c_void_p, C.c_long, C.c_long]),
    "pinc_sim_mg_history": (C.c_long, [C.c_void_p, C.c_void_p, C.c_long]),
    "pinc_sim_mg_levels": (C.c_int, [C.c_void_p]),
    "pinc_sim_mg_shard": (C.c_int, [C.c_void_p]),
    "pinc_sim_spectral_distributed": (C.c_int, [C.c_void_p]),
    "pinc_sim_obj_collected": (C.c_double, [C.c_void_p]),
    "pinc_sim_nspecies": (C.c_int, [C.c_void_p]),
    "pinc_sim_ndims": (C.c_int, [C.c_void_p]),
    "pinc_sim_pop_count": (C.c_long, [C.c_void_p, C.c_int]),
    "pinc_sim_pop_get": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "pinc_sim_pop_set": (C.c_int, [C.c_void_p, C.c_int, C.c_long, C.c_void_p, C.c_void_p]),
    "pinc_sim_grid_shape": (C.c_long, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "pinc_sim_grid_get": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "pinc_sim_grid_set": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "pinc_sim_emigrants": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pinc_sim_species": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "pinc_sim_sync": (C.c_int, [C.c_void_p]),
    "pinc_sim_open_output": (C.c_int, [C.c_void_p]),
    "pinc_sim_write_output": (C.c_int, [C.c_void_p, C.c_double]),
    "pinc_h5_available": (C.c_int, []),
    "pinc_h5_read": (C.c_long, [C.c_char_p, C.c_char_p, C.c_int, C.c_void_p, C.c_long]),
    "pinc_h5_dims": (C.c_int, [C.c_char_p, C.c_char_p, C.c_void_p]),
    "pinc_h5_write": (C.c_int, [C.c_char_p, C.c_char_p, C.c_int, C.c_void_p, C.c_void_p]),
    "pinc_sim_timers": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pinc_sim_timers_reset": (C.c_int, [C.c_void_p]),
    "pinc_sim_total_particles": (C.c_long, [C.c_void_p]),
    "pinc_probe_start": (C.c_int, [C.c_int, C.c_int]),
    "pinc_set_host_transport": (C.c_int, [C.c_void_p]),
    "pinc_comm_stats_start": (C.c_int, [C.c_int]),
    "pinc_comm_stats_read": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "pinc_comm_kind_name": (C.c_char_p, [C.c_int]),
    "pinc_probe_read": (C.c_int, [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int),
                                  C.POINTER(C.c_long)]),
    "pinc_probe_sample": (C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int)]),
}
PROBES = {"gs_pass": 0, "accelerate": 1, "move_classify": 2, "deposit": 3, "residual_sumsq": 4, "spectral": 5, "push": 6,
          "mg_cycle": 7, "push_plain": 8, "push_count": 9, "push_sort": 10}
# probes that split another probe's launches by kind (not separate kernels)
SUB_PROBES = {"push_plain": "push", "push_count": "push", "push_sort": "push"}


def probe_start(kernel: str = "all", max_samples: int = 4096) -> None:
    """Start HIP-event probes on one kernel (PROBES key) or on all of them."""
    k = -1 if kernel == "all" else PROBES[kernel]
    if HOST.pinc_probe_start(k, max_samples):
        raise ValueError(f"bad probe {kernel!r}")


COMM_KINDS = 6


def comm_stats_start(max_calls: int = 16384) -> None:
    """Time and count the library's collectives by kind (pinc_comm.c)."""
    HOST.pinc_comm_stats_start(max_calls)


def comm_stats_read() -> dict:
    """Per collective kind: device ms (over the timed calls), this rank's
    payload bytes, calls, timed calls; {} if statistics were never started."""
    import numpy as _np
    ms, by = _np.zeros(COMM_KINDS), _np.zeros(COMM_KINDS)
    calls, timed = _np.zeros(COMM_KINDS, dtype=_np.int64), _np.zeros(COMM_KINDS, dtype=_np.int64)
    if HOST.pinc_comm_stats_read(ms.ctypes.data, by.ctypes.data, calls.ctypes.data, timed.ctypes.data) < 0:
        return {}
    return {HOST.pinc_comm_kind_name(k).decode(): {"ms": float(ms[k]), "bytes": float(by[k]), "calls": int(calls[k]),
                                                   "timed_calls": int(timed[k])} for k in range(COMM_KINDS)}


PUSH_KIND_NAMES = ("plain", "count", "sort")


def probe_samples(kernel: str) -> list[tuple[float, int]]:
    """(ms, tag) of every recorded launch of a probed kernel, in launch order
    (push: tag = species | kind << 8, PUSH_KIND_NAMES[kind])."""
    out, i = [], 0
    ms, tag = C.c_double(), C.c_int()
    while HOST.pinc_probe_sample(PROBES[kernel], i, C.byref(ms), C.byref(tag)) == 0:
        out.append((ms.value, tag.value))
        i += 1
    return out


def probe_read(kernel: str) -> dict:
    """Mean duration (ms) and algorithmic bytes per probed launch."""
    ms, b, n, launches = C.c_double(), C.c_double(), C.c_int(), C.c_long()
    HOST.pinc_probe_read(PROBES[kernel], C.byref(ms), C.byref(b), C.byref(n), C.byref(launches))
    return {"mean_ms": ms.value, "mean_bytes": b.value, "samples": n.value, "launches": launches.value}
for _n, (_r, _a) in _sigs.items():
    _f = getattr(HOST, _n)
    _f.restype = _r
    _f.argtypes = _a

HIP.pinc_hip_comm_unique_id.restype = C.c_int
HIP.pinc_hip_comm_unique_id.argtypes = [C.c_void_p]
HIP.pinc_hip_error_string.restype = C.c_char_p
HIP.pinc_hip_device_count.argtypes = [C.POINTER(C.c_int)]


def comm_unique_id() -> bytes:
    buf = (C.c_ubyte * PINC_COMM_ID_BYTES)()
    rc = HIP.pinc_hip_comm_unique_id(buf)
    if rc:
        raise RuntimeError(f"ncclGetUniqueId failed: {HIP.pinc_hip_error_string().decode()}")
    return bytes(buf)


def header_symbols(header: Path) -> list[str]:
    """Function names declared in one of the include/*.h headers."""
    import re
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = "\n".join(l for l in text.splitlines() if not l.lstrip().startswith(("typedef", "#")))
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", text, flags=re.M)
    skip = {"if", "for", "while", "return", "sizeof", "defined", "void", "int", "double", "long", "char"}
    return sorted({n for n in names if n not in skip and not n.startswith("__")})
