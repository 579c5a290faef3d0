"""Hash of the sources liblincheck.so is built from (lc_build_id()).

The Makefile bakes it into the library; abi.py recomputes it from the tree
the library is loaded from and refuses a library built from other sources,
so tests, smoke() and bench.py never run a stale binary.
"""
import glob
import hashlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def sources(here=HERE):
    """The inputs of the build, as paths relative to csrc/, sorted."""
    pats = ["*.hip", "*.cpp", "*.h", "Makefile", os.path.join("..", "..", "..", "include", "*.h")]
    rel = set()
    for p in pats:
        for f in glob.glob(os.path.join(here, p)):
            rel.add(os.path.relpath(f, here))
    return sorted(rel)


def build_id(here=HERE):
    h = hashlib.sha256()
    for rel in sources(here):
        h.update(rel.encode() + b"\0")
        with open(os.path.join(here, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(build_id())
