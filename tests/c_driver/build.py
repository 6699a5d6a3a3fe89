"""Compile tests/c_driver/pinc_main.c against the in-tree libpinc.so
(test infrastructure; called by __graft_entry__.build() and the tests)."""
from __future__ import annotations

import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
EXE = HERE / "pinc_main"


def build() -> Path:
    src = HERE / "pinc_main.c"
    lib = ROOT / "pinc_amd" / "lib" / "libpinc.so"
    hdr = [ROOT / "include" / "pinc.h", ROOT / "include" / "pinc_hip.h"]
    if EXE.exists() and all(EXE.stat().st_mtime >= p.stat().st_mtime for p in [src, lib, *hdr]):
        return EXE
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", f"-I{ROOT / 'include'}", str(src), "-o", str(EXE),
                    f"-L{lib.parent}", "-lpinc", f"-Wl,-rpath,{lib.parent}", "-Wl,-rpath,$ORIGIN/../../pinc_amd/lib"],
                   check=True)
    return EXE


if __name__ == "__main__":
    print(build())
