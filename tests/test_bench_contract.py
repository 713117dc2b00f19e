"""CPU checks of bench.py's roofline helpers against the committed profiles/ summaries
(the bench line's `roofline.traffic` and `roofline.valu_issue` come from them)."""
import json
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

KERNELS = {"c2": "void vip::bilateral_kernel<7,", "c3": "void vip::adaptive_kernel<7,",
           "c5": "void vip::bilateral_kernel<15,"}


@pytest.mark.parametrize("cfg", sorted(KERNELS))
def test_pmc_traffic_near_algorithmic_bytes(cfg):
    traffic, src = bench.pmc_traffic(cfg, [KERNELS[cfg]])
    assert src is not None and os.path.exists(os.path.join(ROOT, src))
    geo = bench.CONFIGS[cfg]
    px = geo["width"] * geo.get("frame_height", geo.get("rows_per_rank", 0))
    algorithmic = 6.0 * px  # read RGB8 + write RGB8
    # halo re-reads are partly L2-served: HBM traffic is within [1, 1.5] x the algorithmic bytes
    assert 1.0 <= traffic / algorithmic < 1.5


@pytest.mark.parametrize("cfg", sorted(KERNELS))
def test_valu_issue_roofline_is_consistent(cfg):
    launch_ms = 0.22 if cfg == "c2" else (0.39 if cfg == "c3" else 25.2)
    v = bench.valu_issue(cfg, KERNELS[cfg], launch_ms)
    assert v is not None
    assert v["peak"] == pytest.approx(1024 * 2.4 / 2)
    assert v["achieved"] == pytest.approx(v["wave_instr_per_launch"] / (launch_ms * 1e-3) / 1e9, rel=1e-3)
    assert 0.0 < v["frac"] < 1.0
    assert 0.0 < v["frac_at_load_clock"] <= 1.0


def test_committed_bench_lines_carry_the_contract_fields():
    for cfg in ("c2", "c3", "c4", "c5"):
        with open(os.path.join(ROOT, "profiles", f"r01_{cfg}_bench.json")) as fh:
            line = json.loads(fh.read().strip().splitlines()[-1])
        for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                    "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
            assert key in line, (cfg, key)
        roof = line["roofline"]
        assert roof["frac"] == pytest.approx(roof["achieved"] / roof["peak"], rel=1e-2)
        assert line["cpu_baseline"]["kind"] in ("port", "reference")
