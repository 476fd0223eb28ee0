#!/usr/bin/env python3
"""Hash of the sources libgnpde.so is built from (csrc/*.hip, csrc/*.hpp,
include/gnpde.h, in name order).  The Makefile compiles it into the library
(gnpde_build_id); gnpde._lib.source_hash() recomputes it, so a test and
smoke() can tell whether the loaded library was built from these sources."""
import glob
import hashlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def source_files():
    fs = sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")) + glob.glob(os.path.join(HERE, "csrc", "*.hpp")))
    return fs + [os.path.join(HERE, "..", "include", "gnpde.h")]


def source_hash():
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash())
