#!/usr/bin/env python3
"""Numerics contract table: how far each unpinned numerics
choice can move the outputs.

The library's default (CUDA) profile is bit-exact with the oracle's CUDA profile
(the GPU parity tests). Three of that profile's choices restate nvcc code generation
that no reference artifact pins (the sumk add, the guide-blend contraction, a
correctly rounded exp). For each alternative (oracle.VARIANTS) and for the include/cpp
numerics (CPP profile), this script reports max |delta| and the exact-match / within-1
percentages against the default profile, per filter, on the reference tests' 50x50
random_array inputs and on lenna (C1's image).

Writes profiles/r02_numerics_sensitivity.json. Test infrastructure (uses the oracle).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as o  # noqa: E402


def stats(a, b):
    d = np.abs(a.astype(np.int32) - b.astype(np.int32))
    return {"max_abs": int(d.max()), "exact_pct": round(float((d == 0).mean() * 100), 5),
            "within1_pct": round(float((d <= 1).mean() * 100), 5), "channels": int(d.size)}


def cases():
    img = o.random_image(50, 50)
    guide = o.random_u8(7500)[::-1].copy().reshape(50, 50, 3)
    lenna = np.load(os.path.join(ROOT, "tests", "golden", "lenna_bgr.npz"))["bgr"]
    lguide = np.ascontiguousarray(lenna[::-1, ::-1])
    return {
        "bilateral k9 random_array 50x50": lambda p: o.bilateral(img, 9, profile=p),
        "joint k9 random_array 50x50": lambda p: o.joint_bilateral(img, guide, 9, profile=p),
        "adaptive k9 random_array 50x50": lambda p: o.adaptive(img, 9, profile=p),
        "texture k5 nitr5 random_array 50x50": lambda p: o.texture(img, 5, 5, p),
        "bilateral k11 lenna (C1)": lambda p: o.bilateral(lenna, 11, profile=p, threads=8),
        "bilateral k15 lenna": lambda p: o.bilateral(lenna, 15, profile=p, threads=8),
        "joint k9 lenna": lambda p: o.joint_bilateral(lenna, lguide, 9, profile=p, threads=8),
        "adaptive k15 lenna": lambda p: o.adaptive(lenna, 15, profile=p, threads=8),
        "texture k5 nitr5 lenna": lambda p: o.texture(lenna, 5, 5, p),
    }


def main():
    table = {}
    for name, fn in cases().items():
        base = fn(o.CUDA)
        row = {"include/cpp numerics (CPP profile)": stats(fn(o.CPP), base)}
        for vname, flags in o.VARIANTS.items():
            if vname.startswith(("blend", "exp")) and not name.startswith("texture"):
                continue  # the guide stage exists only in the texture filter
            with o.variant(flags):
                row[vname] = stats(fn(o.CUDA), base)
        table[name] = row
        print(name)
        for k, v in row.items():
            print(f"   {k:38s} max {v['max_abs']}  exact {v['exact_pct']:9.5f}%  <=1 {v['within1_pct']:9.5f}%")
    out = os.path.join(ROOT, "profiles", "r02_numerics_sensitivity.json")
    with open(out, "w") as fh:
        json.dump({"baseline": "oracle CUDA profile == the HIP library's default output (bit-exact, GPU tests)",
                   "table": table}, fh, indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
