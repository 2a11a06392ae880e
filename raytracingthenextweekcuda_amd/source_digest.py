"""The digest that ties librtmi.so, its profiles and the source tree together.

`source_digest(csrc)` hashes every native source of the library (csrc/*.hip, *.cpp, *.h, the
Makefile) and include/rtmi.h, plus the EXTRA compiler flags of the build. The Makefile bakes it
into the library (`rt_kernel_source_sha()`), bench.py stamps it on its line and the rocprofv3
summaries carry it (tools/valu_summary.py, tools/pmc_summary.py), and `_lib.lib()` refuses an
in-tree library whose embedded digest is not the tree's: a stale binary cannot be timed or
profiled under the current sources' name.

Run as a script (the Makefile does): `python3 source_digest.py <csrc dir> [EXTRA flags]`.
"""
from __future__ import annotations

import hashlib
import os
import sys

DIGEST_LEN = 16
SUFFIXES = (".hip", ".cpp", ".h")


def digest_files(csrc: str) -> list:
    """(name, path) of the hashed files, in a fixed order."""
    names = sorted(f for f in os.listdir(csrc)
                   if f.endswith(SUFFIXES) and os.path.isfile(os.path.join(csrc, f)))
    out = [(n, os.path.join(csrc, n)) for n in names]
    out.append(("Makefile", os.path.join(csrc, "Makefile")))
    out.append(("include/rtmi.h", os.path.join(csrc, "..", "..", "include", "rtmi.h")))
    return out


def source_digest(csrc: str, extra: str = "") -> str:
    h = hashlib.sha256()
    for name, path in digest_files(csrc):
        with open(path, "rb") as fh:
            h.update(name.encode() + b"\0" + fh.read() + b"\0")
    # flags that change the binary without changing a file (EXTRA=-DRT_... A/B and ablation builds)
    h.update(b"EXTRA\0" + " ".join(extra.split()).encode())
    return h.hexdigest()[:DIGEST_LEN]


if __name__ == "__main__":
    print(source_digest(sys.argv[1], " ".join(sys.argv[2:])))
