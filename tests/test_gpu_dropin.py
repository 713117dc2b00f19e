"""The C++ drop-in layer (include/cuda/*.hpp, include/impl/*.cuh, DeviceImage,
rocThrust stage overloads) on the GPU, checked against the oracle goldens.

* tests/cpp/dropin_test (built by build()): the reference tests' white-box
  pattern -- subclasses calling impl_->... on thrust::device_vector buffers
  (test/bilateral_filter.cu:9-33, test/bilateral_texture_filter.cu:115-136), the
  blocking public API on DeviceImage buffers (src/device_image.cu:5-52) -- on the
  reference tests' random_array inputs; every output must equal
  tests/golden/oracle_small.npz bit for bit (CUDA numerics, the C++ API's profile).
* samples/vip_benchmark (the sample/benchmark/main.cpp counterpart): its
  per-filter outputs must equal the oracle on the sample's own input.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _run(args, timeout=120):
    exe = args[0]
    assert os.path.exists(exe), f"{exe} missing: run __graft_entry__.build() first"
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_cpp_dropin_whitebox_matches_goldens(tmp_path, goldens):
    out = _run([os.path.join(ROOT, "tests", "cpp", "dropin_test"), GOLDEN, str(tmp_path)])
    assert "0 failures" in out, out

    def load(name, dtype, shape):
        return np.fromfile(tmp_path / f"{name}.bin", dtype=dtype).reshape(shape)

    img = (50, 50, 3)
    checks = {
        "bilateral_k9": ("bilateral_cuda_k9", np.uint8, img),
        "bilateral_k15": ("bilateral_cuda_k15", np.uint8, img),
        "bilateral_k31": ("bilateral_cuda_k31", np.uint8, img),
        "joint_k9": ("joint_cuda_k9", np.uint8, img),
        "adaptive_k9": ("adaptive_cuda_k9", np.uint8, img),
        "adaptive_k15": ("adaptive_cuda_k15", np.uint8, img),
        "texture_k5_n5": ("texture_cuda_k5_n5", np.uint8, (48, 64, 3)),
        "blurred_k5": ("blurred_cuda_k5", np.float32, img),
        "rtv_k5": ("rtv_cuda_k5", np.float32, (50, 50)),
        "guide_k5": ("guide_cuda_k5", np.uint8, img),
        "blurred_k9": ("blurred_cuda_k9", np.float32, img),
        "rtv_k9": ("rtv_cuda_k9", np.float32, (50, 50)),
        "guide_k9": ("guide_cuda_k9", np.uint8, img),
        "gradient_u8_c1": ("gradient_u8_cuda_c1", np.float32, (50, 50)),
        "gradient_u8_c3": ("gradient_u8_cuda_c3", np.float32, (50, 50)),
        "gradient_f32_c1": ("gradient_f32_cuda_c1", np.float32, (50, 50)),
        "gradient_f32_c3": ("gradient_f32_cuda_c3", np.float32, (50, 50)),
    }
    bad = []
    for name, (key, dtype, shape) in checks.items():
        got, want = load(name, dtype, shape), goldens[key]
        # bitwise comparison (f32 stage outputs too)
        if got.tobytes() != want.tobytes():
            bad.append(f"{name}: {int((got != want).sum())} elements differ")
    assert not bad, bad


def test_sample_benchmark_outputs_match_oracle(tmp_path, oracle):
    w, h, k, tk, nitr = 100, 100, 9, 9, 3
    out = _run([os.path.join(ROOT, "samples", "vip_benchmark"), str(w), str(h), "2", str(k), str(tk), str(nitr),
                "--dump", str(tmp_path)])
    inp = np.fromfile(tmp_path / "input.bin", np.uint8).reshape(h, w, 3)
    assert np.array_equal(inp, 100 + oracle.random_u8(w * h * 3, 20).reshape(h, w, 3))
    want = {"bilateral": oracle.bilateral(inp, k), "adaptive": oracle.adaptive(inp, k),
            "texture": oracle.texture(inp, tk, nitr)}
    for name, ref in want.items():
        got = np.fromfile(tmp_path / f"{name}.bin", np.uint8).reshape(h, w, 3)
        assert np.array_equal(got, ref), name
        # the printed checksum is FNV-1a 64 of the output bytes
        hsh = 1469598103934665603
        for b in ref.tobytes():
            hsh = ((hsh ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
        assert f"{hsh:016x}" in out, (name, out)
