"""CPU checks of bench.py's roofline helpers against the committed profiles/ summaries
(the bench line's `roofline.traffic` and `roofline.valu_issue` come from them)."""
import json
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

# exact instantiations (full template signature, as vip_launched_kernels names them) that
# committed PMC summaries hold
KERNELS = {"c3": "void vip::adaptive_kernel<7, 16, true, 4, 512, true>",
           "c5": "void vip::bilateral_kernel<15, 16, false, true, 32, 8, 768, false, 16, false>"}


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


def test_pmc_lookup_needs_the_exact_signature():
    """A summary of another instantiation is stale for a bench line: a prefix, a shorter
    template list (an older build) or another tiling finds nothing."""
    exact = KERNELS["c5"]
    assert bench.pmc_traffic("c5", [exact])[0] is not None
    assert bench.pmc_traffic("c5", ["void vip::bilateral_kernel<15,"]) == (None, None)
    assert bench.pmc_traffic("c5", [exact[:-1] + ", 7>"]) == (None, None)
    # round 3's C2 summary was of the 8-argument template; the benched kernel has 10
    stale = "void vip::bilateral_kernel<7, 16, false, true, 32, 8, 768, false>"
    e, src = bench.pmc_summary("c2", stale, "traffic_bytes")
    assert e is not None and src.endswith("r03_c2_pmc.json")
    assert bench.valu_issue("c2", stale + " ", 0.2) is None
    assert bench.launched([stale, KERNELS["c5"]], "void vip::bilateral_kernel<15,") == KERNELS["c5"]
    assert bench.launched([stale], "void vip::adaptive") is None


def test_committed_lines_cite_a_summary_of_the_kernel_they_timed():
    """Every committed bench line that names its kernel (roofline.kernel_name, round 4 on)
    takes traffic / VALU issue only from a PMC summary holding exactly that kernel."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_bench.json"))):
        lines = [ln for ln in open(f).read().splitlines() if ln.startswith("{")]
        if not lines:
            continue
        roof = json.loads(lines[-1]).get("roofline", {})
        name = roof.get("kernel_name")
        if not name:
            continue
        for src in filter(None, [roof.get("traffic_source"), (roof.get("valu_issue") or {}).get("source")]):
            for one in src.split(", "):
                with open(os.path.join(ROOT, one)) as fh:
                    assert name in json.load(fh)["kernels"], (f, one, name)


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


def test_kernel_busy_isolated_and_union(tmp_path):
    """scripts/kernel_busy.py: launches that overlap another are not 'isolated', and the
    busy time is the union of the launch intervals (frames in flight on two streams)."""
    import subprocess
    rows = [("k", 0, 100), ("k", 50, 150), ("k", 200, 300), ("j", 310, 330)]
    f = tmp_path / "run_kernel_trace.csv"
    f.write_text("Kernel_Name,Start_Timestamp,End_Timestamp\n" + "".join(f"{n},{s},{e}\n" for n, s, e in rows))
    out = tmp_path / "busy.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "kernel_busy.py"), str(f), str(out)], check=True,
                   capture_output=True)
    d = json.loads(out.read_text())
    assert d["launches"] == 4
    assert d["busy_ns_per_launch"] == (150 + 100 + 20) / 4
    assert d["kernels"]["k"]["launches"] == 3 and d["kernels"]["k"]["isolated_launches"] == 1
    assert d["kernels"]["k"]["isolated_mean_us"] == 0.1
    assert d["kernels"]["j"]["isolated_launches"] == 1


def test_committed_lines_time_the_roofline_on_one_stream():
    """With frames in flight (streams > 1) the roofline's launch duration is the single-
    stream one, which the committed rocprofv3 isolated launches must agree with (<= 3 %)."""
    for cfg, kern in (("c2", "void vip::bilateral_kernel<7,"), ("c4", "void vip::texture_guide_fused_kernel<2,")):
        line = json.load(open(os.path.join(ROOT, "profiles", f"r02_{cfg}_bench.json")))
        busy = json.load(open(os.path.join(ROOT, "profiles", f"r02_{cfg}_busy.json")))
        assert line["streams"] == 2 and line["frame_ms_in_flight"] <= line["kernel_ms"]
        iso = [v["isolated_mean_us"] for n, v in busy["kernels"].items() if n.startswith(kern)][0]
        r = line["roofline"]
        launch_ms = r["avg_launch_ms"] if cfg == "c2" else \
            [k["avg_launch_ms"] for k in (r["dominant"], r["other"]) if "guide" in k["kernel"]][0]
        assert abs(iso / 1e3 - launch_ms) / launch_ms < 0.03, (cfg, iso, launch_ms)


# A kernel's own begin-to-end duration includes its drain: a launch ends when its slowest
# workgroup does, and the XCDs hold clocks up to ~5 % apart under load,
# so the last round's workgroups on the fast XCDs idle while the slow XCD finishes. With two
# frames in flight the next frame fills those CUs. Measured C2 (kernel-stamped launch against
# ms_per_step): 0.1757 / 0.1737 (x 1.012, profiles/r06a_c2_bench.json) and 0.1774 / 0.1687
# (x 1.052, profiles/r06b_c2_bench.json). So the duration behind frac may exceed the step by
# that drain, never by launch gaps: BENCH_r05's one-stream event span (0.1821 against 0.176,
# x 1.035, with a 0.1705-ms kernel) timed the gaps between launches as well.
DRAIN_ALLOWANCE = 1.06


def roofline_duration_fits_a_step(line) -> bool:
    """The kernel duration behind `roofline.frac` (avg_launch_ms, per frame) fits in the
    measured step: <= ms_per_step x frames per launch, up to the drain the
    other stream fills (DRAIN_ALLOWANCE). It holds for kernels that fill the chip (C2, C3,
    C5, C4's stages); C1's 512^2 launches each hold a fraction of the CUs and run side by
    side, which `roofline.in_flight` reports."""
    r = line["roofline"]
    fpl = r.get("frames_per_launch", 1)
    if "dominant" in r:  # C4: a stage launch against the frame's step (10 launches per frame)
        return r["avg_launch_ms"] <= line["ms_per_step"]
    return r["avg_launch_ms"] <= line["ms_per_step"] * fpl * DRAIN_ALLOWANCE


def test_roofline_duration_rule():
    ok = dict(ms_per_step=0.1687, roofline=dict(avg_launch_ms=0.1774))  # r06b: kernel-stamped
    gaps = dict(ms_per_step=0.1687, roofline=dict(avg_launch_ms=0.1829))  # r06b's one-stream span
    assert roofline_duration_fits_a_step(ok) and not roofline_duration_fits_a_step(gaps)


def test_committed_lines_divide_by_a_kernel_duration_that_fits_a_step():
    """Every committed N = 1 line timed with vip_kernel_timing (kernel-stamped events) of a
    chip-filling config: the duration behind frac fits in ms_per_step."""
    import glob
    lines = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_c[2345]_bench.json"))) + \
            sorted(glob.glob(os.path.join(ROOT, "BENCH_r*.json"))):
        try:
            line = json.load(open(f))
        except ValueError:
            continue
        line = line.get("parsed", line)
        if isinstance(line, dict) and line.get("n_gpus") == 1 and "launch_timing" in line.get("roofline", {}):
            lines.append((f, line))
    if not lines:
        pytest.skip("no committed line timed with vip_kernel_timing yet")
    for f, line in lines:
        assert roofline_duration_fits_a_step(line), (f, line["roofline"]["avg_launch_ms"], line["ms_per_step"])


# what one N-GPU bench line may take on the device, startup excluded: the driver runs
# N = 1, 2, 4, 8 back to back on one node, so each line must stay well inside its limit
MULTI_GPU_LINE_BUDGET_S = 60.0


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_multi_gpu_trial_wall_time_is_bounded(cfg):
    """The N > 1 trial: every form the trial times, with the step times
    of the loopback rehearsals at that N (profiles/r0*_<cfg>_loopback<N>_bench.json), or the
    N = 1 line's step split N ways (C4: a 2160-row slab per rank, the N = 1 step) where no
    rehearsal exists, fits MULTI_GPU_LINE_BUDGET_S per line. The N = 8 constants (free CUs,
    frames per RCCL group) are re-tuned only from the driver's own xGMI lines."""
    import glob

    def line(path):  # the JSON line (rehearsal files carry RCCL's banner before it)
        return json.loads([x for x in open(path) if x.startswith("{")][-1])
    n1 = line(os.path.join(ROOT, "profiles", f"r05_final_{cfg}_bench.json"))["ms_per_step"]
    for n in (2, 4, 8):
        got = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r0*_{cfg}_loopback{n}_bench.json")))
        step = line(got[-1])["ms_per_step"] if got else (n1 if cfg == "c4" else n1 / n)
        step = max(step, n1 if cfg == "c4" else n1 / n)  # never below linear
        t = bench.multi_gpu_wall_estimate_s(cfg, n, step * 1.5)  # xGMI exchange slower than loopback: 1.5x
        assert t < MULTI_GPU_LINE_BUDGET_S, (cfg, n, step, t)
    assert len(bench.native_forms(bench.TRIAL_STREAMS, False)) == 48
    assert len(bench.native_forms(bench.TRIAL_STREAMS, True)) == 9


def test_halo_batches_keep_buffers_on_one_stream():
    """bench.py N > 1 native path: frame i in batch i // B on stream (i // B) % S. For
    every batch size it may choose, each buffer (i % NBUF) always meets the same stream,
    and every batch lies on one stream, for any frame count and any phase boundaries."""
    for S in (1, 2, 3, 4, 6):
        for B in bench.halo_batches(S):
            seen = {}
            for i in range(10 * bench.NBUF * B):
                st = (i // B) % S
                assert seen.setdefault(i % bench.NBUF, st) == st
    assert bench.halo_batches(2) == [1, 2, 3, 6] and bench.halo_batches(3) == [1, 2, 4]


# --- `python bench.py --gpus N` starts its own N ranks -------------
PROBE = r'''
import json, os, sys, time
rank = os.environ["RANK"]
with open(os.path.join(sys.argv[1], f"rank{rank}.json"), "w") as fh:
    json.dump({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                                              "HSA_ENABLE_IPC_MODE_LEGACY")} | {"argv": sys.argv[1:]}, fh)
if sys.argv[2] == "sleep":
    time.sleep(120)
sys.exit(int(sys.argv[2]) if rank == "1" and sys.argv[2] != "sleep" else 0)
'''


def test_rank_launch_argv_is_the_drivers_form():
    cmd = bench.rank_launch_argv(4, ["--gpus", "4", "--config", "c5"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--config", "c5"]


def _probe(tmp_path):
    script = tmp_path / "probe.py"
    script.write_text(PROBE)
    return str(script)


def test_launch_ranks_env_and_status(tmp_path):
    script = _probe(tmp_path)
    rc = bench.launch_ranks(2, [str(tmp_path), "0"], timeout_s=120, script=script)
    assert rc == 0
    envs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in (0, 1)]
    for r, e in enumerate(envs):
        assert e["RANK"] == str(r) and e["LOCAL_RANK"] == str(r) and e["WORLD_SIZE"] == "2"
        assert e["MASTER_ADDR"] == "127.0.0.1" and int(e["MASTER_PORT"]) > 0
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert e["argv"] == [str(tmp_path), "0"]
    # one failing rank fails the run
    assert bench.launch_ranks(2, [str(tmp_path), "3"], timeout_s=120, script=script) != 0


def test_launch_ranks_timeout_ends_every_rank(tmp_path):
    import time
    script = _probe(tmp_path)
    t0 = time.monotonic()
    rc = bench.launch_ranks(2, [str(tmp_path), "sleep"], timeout_s=15, script=script)
    assert rc == 124 and time.monotonic() - t0 < 60
    # the ranks were started (they wrote their env) and are gone now
    assert (tmp_path / "rank0.json").exists() and (tmp_path / "rank1.json").exists()


def test_bench_gpus_2_from_a_plain_shell_launches_ranks():
    """`python bench.py --gpus 2` without WORLD_SIZE starts two ranks through torchrun; on
    this GPU-less host they fail, and that failure is the command's status (no exit at the
    launch check, no hang)."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--launch-timeout", "240"], capture_output=True, text=True, env=env, timeout=300)
    assert "starting 2 ranks" in r.stderr
    assert "torch.distributed.run" in r.stderr
    assert r.returncode not in (0, 124)


def test_default_multi_gpu_run_is_one_plain_launch(monkeypatch):
    """`python bench.py --gpus N` starts the ranks ONCE with the arguments it was given: no
    graph-capture attempt, no second HIP runtime or RCCL in a rank."""
    calls = []
    monkeypatch.setattr(bench, "launch_ranks", lambda n, argv, timeout_s=0, script=None: calls.append((n, argv)) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and calls == [(8, ["--gpus", "8"])]
    assert not any("graph" in a for a in calls[0][1])
    for gone in ("preload_system_rocm", "launch_with_graph_attempt", "SYSTEM_ROCM"):
        assert not hasattr(bench, gone)
    with pytest.raises(SystemExit):  # and no --graph option to ask for it
        monkeypatch.setattr(sys, "argv", ["bench.py", "--graph"])
        bench.parse()


def test_native_trial_forms_keep_buffers_on_one_stream():
    """The N > 1 native trial's forms (streams S, split, frames per RCCL group B, shared):
    every S of TRIAL_STREAMS appears, each (S, B) keeps buffer i % NBUF on one stream, the
    texture filter has no split form, and --batch restricts B."""
    forms = bench.native_forms(bench.TRIAL_STREAMS, texture=False)
    assert {f[0] for f in forms} == set(bench.TRIAL_STREAMS)
    assert all(bench.NBUF % (s * b) == 0 for s, _, b, _ in forms)
    assert {(s, sp) for s, sp, _, _ in forms} == {(s, sp) for s in bench.TRIAL_STREAMS for sp in (True, False)}
    # shared launches: only after the exchange (no split) and for more than one frame
    assert all(not sp and b > 1 for _, sp, b, sh in forms if sh is not None)
    assert {(s, b, sh) for s, _, b, sh in forms if sh is not None} == {
        (s, b, fc) for s in bench.TRIAL_STREAMS for b in bench.halo_batches(s) if b > 1 for fc in bench.SHARED_FREE_CUS}
    tex = bench.native_forms([2], texture=True)
    assert all(not sp and sh is None for _, sp, _, sh in tex)
    assert len(set(forms)) == len(forms)
    assert {b for _, _, b, _ in bench.native_forms(bench.TRIAL_STREAMS, texture=False, batches=[3])} == {3}


def test_single_gpu_trial_uses_the_multi_gpu_grid():
    """N = 1 (plain and adaptive) is timed over the same streams x frames-per-launch grid
    as the N > 1 trial, B = 1 included."""
    one = bench.single_gpu_forms(bench.TRIAL_STREAMS)
    assert set(one) == {(s, b) for s, _, b, _ in bench.native_forms(bench.TRIAL_STREAMS, texture=False)}
    assert (2, 1) in one and (2, 6) in one and (4, 3) in one
    assert bench.single_gpu_forms([2], [1]) == [(2, 1)]


class _FakeShard:
    def __init__(self, count, user_rank, device, bus):
        self.i = dict(count=count, user_rank=user_rank, device=device, pci_bus_id=bus)

    def comm_info(self):
        return dict(self.i)


def test_rccl_evidence_flags_what_is_not_an_n_gpu_run(monkeypatch):
    """The line's `rccl` block: RCCL's own count / user rank / device per rank, and the
    problems that make a line invalid (a communicator of another size, two ranks on one
    device, communicators of one rank that disagree)."""
    import various_image_processings_amd.sharded as sh
    monkeypatch.setattr(sh, "rccl_version", lambda: 22606)
    ok = bench.rccl_evidence([_FakeShard(1, 0, 0, "0000:05:00.0")] * 2, 0, 1, 1)
    assert ok["problems"] == [] and ok["count"] == 1 and ok["distinct_devices"] == 1 and ok["rccl_version"] == 22606
    bad = bench.rccl_evidence([_FakeShard(1, 0, 0, "0000:05:00.0")], 0, 1, 8)
    assert bad["problems"] and "expected 8" in bad["problems"][0]
    mixed = bench.rccl_evidence([_FakeShard(1, 0, 0, "b"), _FakeShard(2, 0, 0, "b")], 0, 1, 1)
    assert any("disagree" in p for p in mixed["problems"])

    class _Broken:
        def comm_info(self):
            raise RuntimeError("ncclCommCount failed")
    broken = bench.rccl_evidence([_Broken()], 0, 1, 1)  # no raise: the peers must reach the gather
    assert any("comm_info failed" in p for p in broken["problems"])


def test_launched_prefers_the_multi_frame_form():
    """A shared launch's kernel (`..._frames_kernel<`) names the line's kernel when present;
    otherwise the one-frame kernel with the prefix; None when neither launched."""
    one = "void vip::bilateral_kernel<7, 16, false, true, 32, 4, 768, false, 64, false>"
    frames = "void vip::bilateral_frames_kernel<7, 16, false, true, 32, 4, 768, false, 64, false>"
    assert bench.launched([one, frames], "void vip::bilateral_kernel<7,") == frames
    assert bench.launched([one], "void vip::bilateral_kernel<7,") == one
    assert bench.launched(["void vip::adaptive_kernel<7, 16, true, 4, 512, true>"],
                          "void vip::bilateral_kernel<7,") is None


ISO_KERNELS = {"c2": ["void vip::bilateral_kernel<7, 16, false, true, 32, 8, 768, false, 16, false>"],
               "c3": ["void vip::adaptive_kernel<7, 16, true, 4, 512, true>"],
               "c4": ["void vip::bilateral_kernel<4, 16, true, true, 32, 8, 32, true, 16, true>"],
               "c5": ["void vip::bilateral_kernel<15, 16, false, true, 32, 8, 768, false, 16, false>"]}


def test_c1_shared_launch_sample():
    """C1's line takes 3 frames per shared launch on 4 streams: its sample is of that
    multi-frame kernel, profiled on one stream with the tiling planned for 4 frames in flight
    (bench.py --batch 3 --frames-in-flight 4), and its PMC summary holds the same kernel."""
    kern = "void vip::bilateral_frames_kernel<5, 16, false, true, 32, 4, 768, false, 64, false>"
    s = bench.isolated_sample("c1", kern)
    assert s is not None and s["launches"] >= 200
    assert bench.valu_issue("c1", kern, s["mean_us"] / 1e3) is not None


@pytest.mark.parametrize("cfg", sorted(ISO_KERNELS))
def test_isolated_launch_samples_are_large_enough(cfg):
    """the launch duration behind each headline roofline rests on a
    committed single-stream rocprofv3 sample (profiles/r0N_<cfg>_isolated.csv, via
    scripts/isolated_sample.py) of at least 200 launches of the exact instantiation, and the
    same round's committed line's live launch duration agrees with it to 3 %."""
    for kern in ISO_KERNELS[cfg]:
        s = bench.isolated_sample(cfg, kern)
        assert s is not None and s["launches"] >= 200, (cfg, kern, s)
        assert s["min_us"] <= s["median_us"] <= s["max_us"]
    # the committed line of the same round as the newest sample (profiles/rNN_<cfg>_bench.json)
    rnd = os.path.basename(bench.isolated_sample(cfg, ISO_KERNELS[cfg][0])["source"]).split("_")[0]
    line = json.loads(open(os.path.join(ROOT, "profiles", f"{rnd}_{cfg}_bench.json")).read().strip().splitlines()[-1])
    r = line["roofline"]
    if cfg == "c4":  # the JBF launch (the guide stage's instantiation carries its argument list)
        launch_ms = [k["avg_launch_ms"] for k in (r["dominant"], r["other"]) if "joint" in k["kernel"]][0]
    else:
        launch_ms = r["avg_launch_ms"]
    iso = bench.isolated_sample(cfg, ISO_KERNELS[cfg][0])["mean_us"] / 1e3
    assert abs(iso - launch_ms) / launch_ms < 0.03, (cfg, iso, launch_ms)
    # a guide-stage sample exists too (its name carries the argument list in the trace)
    if cfg == "c4":
        import csv
        rows = list(csv.DictReader(open(os.path.join(ROOT, "profiles", "r05_c4_isolated.csv"))))
        assert sum(1 for x in rows if x["kernel"].startswith("void vip::texture_guide_fused_kernel<2, false>")) >= 200


def test_isolated_sample_script(tmp_path):
    """scripts/isolated_sample.py keeps the last N non-overlapping launches per kernel above
    the duration floor."""
    import subprocess
    rows = [("k", i * 100, i * 100 + 50) for i in range(10)] + [("j", 2000, 2001), ("k", 2010, 2100), ("k", 2050, 2150),
                                                                ("z(int)", 2200, 2900)]
    f = tmp_path / "t.csv"
    f.write_text("Kernel_Name,Start_Timestamp,End_Timestamp\n" + "".join(f"{n},{s},{e}\n" for n, s, e in rows))
    out = tmp_path / "o.csv"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "isolated_sample.py"), str(f), str(out), "--last", "4",
                    "--min-us", "0.01", "--prefix", "k"], check=True, capture_output=True)
    import csv
    got = list(csv.DictReader(open(out)))
    assert [int(r["index"]) for r in got if r["kernel"] == "k"] == [6, 7, 8, 9]  # overlapping pair dropped
    assert all(int(r["duration_ns"]) == 50 for r in got if r["kernel"] == "k")
    assert not [r for r in got if r["kernel"] in ("j", "z")]  # below the floor; another prefix


def test_aligned_phases_make_whole_batches():
    """bench.py flushes a batch when (i + 1) % B == 0; every phase (trial form, warm-up,
    timed steps) starts at align(i), a multiple of NBUF, so with a phase length that B
    divides every batch has exactly B frames -- the PMC and launch samples of a shared
    launch then always carry B frames."""
    for S in (1, 2, 3, 4):
        for B in bench.halo_batches(S):
            for start in (0, 5, 13, 1001):
                i0 = bench.align(start)
                assert i0 % bench.NBUF == 0 and 0 <= i0 - start < bench.NBUF
                sizes, pending = [], []
                for i in range(i0, i0 + 12 * B):
                    pending.append(i)
                    if (i + 1) % B == 0:
                        sizes.append(len(pending))
                        pending = []
                assert not pending and set(sizes) == {B}


def test_pmc_summary_records_frames_per_launch(tmp_path):
    """scripts/pmc_summary.py --frames-per-launch B marks the multi-frame kernels of a
    `bench.py --batch B` pass, and bench.py divides their counts and bytes per frame."""
    import subprocess
    d = tmp_path / "pmc"
    (d / "p1").mkdir(parents=True)
    rows = [("void vip::bilateral_frames_kernel<5, 16>(vip::StencilArgs)", "SQ_INSTS_VALU", 3000.0),
            ("void vip::bilateral_kernel<5, 16>(vip::StencilArgs)", "SQ_INSTS_VALU", 1000.0),
            ("void vip::bilateral_frames_kernel<5, 16>(vip::StencilArgs)", "FETCH_SIZE", 30.0),
            ("void vip::bilateral_frames_kernel<5, 16>(vip::StencilArgs)", "WRITE_SIZE", 60.0)]
    (d / "p1" / "run_counter_collection.csv").write_text(
        "Kernel_Name,Counter_Name,Counter_Value\n" + "".join(f'"{k}",{c},{v}\n' for k, c, v in rows))
    out = tmp_path / "r99_cx_pmc.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), str(d), str(out),
                    "--frames-per-launch", "3"], check=True, capture_output=True)
    k = json.loads(out.read_text())["kernels"]
    assert k["void vip::bilateral_frames_kernel<5, 16>"]["frames_per_launch"] == 3
    assert "frames_per_launch" not in k["void vip::bilateral_kernel<5, 16>"]
    e = k["void vip::bilateral_frames_kernel<5, 16>"]
    assert e["traffic_bytes"] == (2 * 30 + 60) * 1024
