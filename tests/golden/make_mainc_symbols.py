"""Generate tests/golden/mainc_symbols.json: the library symbols the
reference's src/main.c needs at link time.

Run in the survey container only (it reads /root/reference/src/main.c as
text; the GPU box has no /root/reference).  The JSON is data: identifiers of
the reference's main.c that are called, or passed to select() as selectors
or to gHaloOp as slice operators, minus
  * MPI_* and gsl_* (the MPI runtime and GSL, which a PINC build links itself),
  * what main.c defines (main, regular, regular_set) and its local function
    pointers (run, acc, distr, ...),
  * C keywords and the select() macro, which expands to selectInner
    (io.h:105) -- selectInner is listed instead.

    python tests/golden/make_mainc_symbols.py [path/to/main.c]
"""
import json
import re
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/main.c")


def symbols(text: str) -> dict:
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    text = re.sub(r'"(?:\\.|[^"\\])*"', '""', text)
    defined = set(re.findall(r"^\w[\w\s\*]*?\b(\w+)\s*\([^;]*?\)\s*\{", text, flags=re.M))
    # local function pointers: void (*name)() / void *(*name)()
    locals_ = set(re.findall(r"\(\s*\*\s*(\w+)\s*\)\s*\(", text))
    keywords = {"if", "for", "while", "return", "sizeof", "switch", "select", "void"}
    called = set(re.findall(r"\b([A-Za-z_]\w*)\s*\(", text))
    # arguments of select(...) and the slice operators given to gHaloOp
    selectors = set()
    for m in re.finditer(r"\bselect\s*\(([^;]*?)\)\s*;", text, flags=re.S):
        selectors.update(a for a in re.findall(r"\b(\w+_set)\b", m.group(1)))
    ops = set(re.findall(r"gHaloOp\s*\(\s*(\w+)", text))
    skip = keywords | defined | locals_
    funcs = {n for n in called if n not in skip and not n.startswith(("MPI_", "gsl_"))}
    funcs |= {"selectInner"} if re.search(r"\bselect\s*\(", text) else set()
    out = {
        "source": "src/main.c",
        "functions": sorted(funcs),
        "selectors": sorted(selectors - defined),
        "slice_ops": sorted(ops),
        "excluded": {
            "defined_in_main_c": sorted(defined),
            "local_function_pointers": sorted(locals_),
            "mpi": sorted(n for n in called if n.startswith("MPI_")),
            "gsl": sorted(n for n in called if n.startswith("gsl_")),
        },
    }
    return out


if __name__ == "__main__":
    data = symbols(SRC.read_text())
    (HERE / "mainc_symbols.json").write_text(json.dumps(data, indent=1) + "\n")
    print(json.dumps(data, indent=1))
