"""Build stamp: which sources the shipped libraries were built from.

`__graft_entry__.build()` writes build_info.json beside the libraries: a sha256 over every
source the libraries compile (the HIP kernels, the C ABI, the headers, the build files), the
sha256 of each built library and the compiler. On a GPU box that runs the pushed tree without
building, `check()` recomputes both and says whether the loaded libraries are the ones built
from the sources that travelled with them (bench.py puts that in its line as `build`)."""
from __future__ import annotations

import glob
import hashlib
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
INFO = os.path.join(HERE, "build_info.json")
LIBS = ("libvip_hip.so", "libvip_shard.so")


def source_files() -> list:
    pats = ["various_image_processings_amd/csrc/*.hip", "various_image_processings_amd/csrc/*.hpp",
            "various_image_processings_amd/csrc/*.cpp", "various_image_processings_amd/csrc/*.inc",
            "various_image_processings_amd/csrc/Makefile", "include/*.h", "include/cuda/*.hpp",
            "include/impl/*.cuh", "CMakeLists.txt"]
    return sorted({os.path.relpath(f, ROOT) for p in pats for f in glob.glob(os.path.join(ROOT, p))})


def _sha(paths) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(p.encode())
        with open(os.path.join(ROOT, p), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _lib_sha(name: str):
    p = os.path.join(HERE, name)
    return _sha([os.path.relpath(p, ROOT)]) if os.path.exists(p) else None


def write(compiler: str = "") -> dict:
    import datetime
    info = dict(sources_sha256=_sha(source_files()), sources=len(source_files()),
                libs={n: _lib_sha(n) for n in LIBS}, compiler=compiler,
                built_utc=datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds"))
    with open(INFO, "w") as fh:
        json.dump(info, fh, indent=1)
    return info


def check() -> dict:
    """The stamp against the tree as it is now: sources_match (the sources the stamp names
    are these) and libs_match (the libraries on disk are the ones it built)."""
    if not os.path.exists(INFO):
        return dict(stamp=None, note="no build_info.json: the libraries were not built by __graft_entry__.build()")
    info = json.load(open(INFO))
    now_src = _sha(source_files())
    libs_now = {n: _lib_sha(n) for n in LIBS}
    return dict(built_utc=info.get("built_utc"), compiler=info.get("compiler"),
                sources_sha256=now_src[:16], sources_match=now_src == info.get("sources_sha256"),
                libs_match=all(libs_now[n] is not None and libs_now[n] == info.get("libs", {}).get(n) for n in LIBS))
