"""Build the in-tree native libraries of the MI355X PINC hot path.

    pinc_amd/lib/libpinc_hip.so   gfx950 kernels + C ABI (include/pinc_hip.h)
    pinc_amd/lib/libpinc.so       host operator surface in C (include/pinc.h)

Run ``python -m pinc_amd.build``; ``__graft_entry__.build()`` also builds the
CPU checker under oracle/ (test infrastructure, not part of this package).
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "pinc_amd" / "csrc"
HOST = ROOT / "pinc_amd" / "host"
# PINC_LIBDIR / PINC_HIP_DEFINES: a variant build (kernel experiments) next to
# the default one, e.g. PINC_LIBDIR=pinc_amd/lib_i2 PINC_HIP_DEFINES="-DPINC_PUSH_ITEMS=2"
LIB = Path(os.environ.get("PINC_LIBDIR") or ROOT / "pinc_amd" / "lib").resolve()
OBJ = ROOT / "build" / ("obj" if LIB == (ROOT / "pinc_amd" / "lib").resolve() else "obj_" + LIB.name)
INC = ROOT / "include"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PINC_ARCH", "gfx950")
# -ffp-contract=off: the kernels reproduce the reference's fp64 association
# order; a fused multiply-add would change the rounding.
# build_flags.txt records what a library was built with (arch, compiler,
# defines); a change of any of them rebuilds.  A variant library (PINC_LIBDIR)
# keeps its defines when rebuilt without PINC_HIP_DEFINES in the environment;
# the default library never inherits defines: it is built with exactly what
# the environment says (none, normally), so bench and tests cannot silently
# run a variant kernel.
STAMP = LIB / "build_flags.txt"
VARIANT = LIB != (ROOT / "pinc_amd" / "lib").resolve()


def _read_stamp() -> dict:
    try:
        return json.loads(STAMP.read_text())
    except (OSError, ValueError):
        return {}


DEFINES = os.environ.get("PINC_HIP_DEFINES")
if DEFINES is None:
    DEFINES = _read_stamp().get("defines", "") if VARIANT else ""
DEFINES = DEFINES.strip()


def stamp() -> dict:
    """What the libraries in LIB are (to be) built with."""
    return {"arch": ARCH, "hipcc": HIPCC, "defines": DEFINES}
HIP_FLAGS = ["-std=c++17", "-O3", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fPIC",
             "-munsafe-fp-atomics", f"-I{INC}", f"-I{CSRC}", *DEFINES.split()]
C_FLAGS = ["-std=c11", "-O2", "-fPIC", "-Wall", "-ffp-contract=off", f"-I{INC}", f"-I{HOST}"]

HIP_SRC = ["runtime.hip", "k_particles.hip", "k_grid.hip", "k_mg.hip", "k_spectral.hip", "k_objects.hip"]
C_SRC = ["pinc_core.c", "pinc_boot.c", "pinc_comm.c", "pinc_grid.c", "pinc_pop.c", "pinc_pusher.c", "pinc_mg.c", "pinc_spectral.c", "pinc_regular.c", "pinc_h5.c", "pinc_obj.c"]


def _run(cmd: list[str], log: Path | None = None) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if log is not None:
        log.write_text(r.stderr)


def _resources_log(src: str) -> Path:
    """The compiler's per-kernel resource report of one HIP source (VGPRs,
    spills, LDS, occupancy: -Rpass-analysis=kernel-resource-usage)."""
    return LIB / f"{src}.resources.txt"


def kernel_resources(lib: Path | None = None) -> dict:
    """{kernel (mangled): {"vgprs", "vgpr_spill", "sgpr_spill", "occupancy", "lds"}} from the
    resource reports the last build wrote next to the libraries."""
    import re
    out = {}
    for f in HIP_SRC:
        p = (lib or LIB) / f"{f}.resources.txt"
        if not p.exists():
            continue
        cur = None
        for line in p.read_text().splitlines():
            m = re.search(r"remark: Function Name: (\S+)", line)
            if m:
                cur = out.setdefault(m.group(1), {"source": f})
                continue
            m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)",
                          line)
            if m and cur is not None:
                key = {"VGPRs": "vgprs", "VGPRs Spill": "vgpr_spill", "SGPRs Spill": "sgpr_spill",
                       "Occupancy [waves/SIMD]": "occupancy", "LDS Size [bytes/block]": "lds"}[m.group(1)]
                cur[key] = int(m.group(2))
    return out


def _newer(src: Path, dst: Path, deps: list[Path]) -> bool:
    if not dst.exists():
        return True
    t = dst.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


def _up_to_date(libs: list[Path], inputs: list[Path]) -> bool:
    """The libraries exist, are newer than every source and header, and were
    built with this arch, compiler and defines.  (The object directory is not consulted: it
    does not travel to the GPU box, where the libraries are used as built.)"""
    if not all(p.exists() for p in libs):
        return False
    if _read_stamp() != stamp():
        return False
    t = min(p.stat().st_mtime for p in libs)
    return all(p.stat().st_mtime <= t for p in inputs)


def build(verbose: bool = False, jobs: int = 8) -> dict:
    hip_deps = [INC / "pinc_hip.h", CSRC / "common.h"]
    c_deps = [INC / "pinc.h", INC / "pinc_hip.h", HOST / "pinc_internal.h"]
    libhip = LIB / "libpinc_hip.so"
    libhost = LIB / "libpinc.so"
    out = {"libpinc_hip": str(libhip), "libpinc": str(libhost)}
    inputs = [CSRC / f for f in HIP_SRC] + [HOST / f for f in C_SRC] + hip_deps + c_deps
    if _up_to_date([libhip, libhost], inputs):
        if verbose:
            print(out)
        return out
    LIB.mkdir(parents=True, exist_ok=True)
    OBJ.mkdir(parents=True, exist_ok=True)
    flags_changed = _read_stamp() != stamp()
    jobs_list = []
    for f in HIP_SRC:
        src, obj = CSRC / f, OBJ / (f + ".o")
        if flags_changed or _newer(src, obj, hip_deps) or not _resources_log(f).exists():
            jobs_list.append(([HIPCC, *HIP_FLAGS, "-Rpass-analysis=kernel-resource-usage", "-c", str(src), "-o",
                               str(obj)], _resources_log(f)))
    for f in C_SRC:
        src, obj = HOST / f, OBJ / (f + ".o")
        if _newer(src, obj, c_deps):
            jobs_list.append((["gcc", *C_FLAGS, "-c", str(src), "-o", str(obj)], None))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda j: _run(*j), jobs_list))
    hip_objs = [str(OBJ / (f + ".o")) for f in HIP_SRC]
    c_objs = [str(OBJ / (f + ".o")) for f in C_SRC]
    _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", str(libhip), *hip_objs,
          "-L/opt/rocm/lib", "-lrccl", "-lrocfft", "-Wl,-rpath,/opt/rocm/lib"])
    _run(["gcc", "-shared", "-o", str(libhost), *c_objs, f"-L{LIB}", "-lpinc_hip", "-lm", "-ldl",
          "-Wl,-rpath,$ORIGIN"])
    STAMP.write_text(json.dumps(stamp()) + "\n")
    if verbose:
        print(out)
    return out


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
