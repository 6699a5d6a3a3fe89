"""Compile the C callers under tests/c_driver/ (pinc_main.c: regular()
through select(); pinc_objmain.c: main.c's object loop through the
reference's object API; pinc_mainc.c: main.c's main() and regular() call for
call) against the in-tree libpinc.so (test
infrastructure; called by __graft_entry__.build() and the tests)."""
from __future__ import annotations

import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
EXE = HERE / "pinc_main"


def build(name: str = "pinc_main") -> Path:
    src = HERE / f"{name}.c"
    exe = HERE / name
    lib = ROOT / "pinc_amd" / "lib" / "libpinc.so"
    hdr = [ROOT / "include" / h for h in ("pinc.h", "pinc_hip.h", "core.h", "pusher.h", "multigrid.h", "spectral.h")]
    if exe.exists() and all(exe.stat().st_mtime >= p.stat().st_mtime for p in [src, lib, *hdr]):
        return exe
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", f"-I{ROOT / 'include'}", str(src), "-o", str(exe),
                    f"-L{lib.parent}", "-lpinc", f"-Wl,-rpath,{lib.parent}", "-Wl,-rpath,$ORIGIN/../../pinc_amd/lib"],
                   check=True)
    return exe


if __name__ == "__main__":
    print(build())
    print(build("pinc_objmain"))
    print(build("pinc_mainc"))
