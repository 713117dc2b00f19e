#!/usr/bin/env python3
"""Benchmark of the MI355X bilateral-filter family (BASELINE.json metric:
"Mpixels/sec bilateral r=7 on 4K RGB; % HBM roofline; 1/2/4/8-GPU scaling").

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]

One step = one filter application over each rank's row slab of a frame that is
row-sharded across the N GPUs (one process per GPU, torch.distributed over
RCCL/xGMI). `python bench.py --gpus N` with N > 1 starts the N ranks itself (a child
`python -m torch.distributed.run --nproc-per-node N ... bench.py`, before anything
touches the GPU) and exits with its status; run under torch.distributed.run directly,
each process is one rank. Each step the ranks exchange their r-row halos with the row
neighbours only (include/vip_shard.h: ncclSend/ncclRecv on the library's own RCCL
communicators, one per stream), then filter their own rows.

  c2 (default) bilateral r=7 (ksize 15, sigma_space 10, sigma_color 30) on the
     3840x2160 RGB8 frame, its rows split over the N ranks (strong scaling: BASELINE
     config 2 at every N); the line also reports the weak-scaling figure (a 2160-row
     slab per rank of an (N*2160)x3840 frame) under "weak".
  c3 adaptive bilateral r=7, same geometry (BASELINE config 3).
  c4 bilateral texture filter k=5, nitr=5 on 3840x2160 per rank (BASELINE config
     4); N>1 row-shards an (N*2160)x3840 frame with one 45-row halo exchange per
     frame (vip_shard_create_texture; sharded.ShardedTexture over torch P2P for the
     gloo rehearsal).
  c5 bilateral r=15 (ksize 31) on ONE 16384x16384 frame row-tiled over the N
     GPUs (strong scaling; BASELINE config 5).

Inputs are synthetic (test/random_array-style uniform u8), resident in HBM before
timing; 12 distinct input/output slabs rotate so the working set exceeds the
256 MB Infinity Cache. Rank 0 prints ONE JSON line. The roofline object is for
the dominant kernel, timed with HIP events on the stream it runs on, beside the
committed single-stream rocprofv3 launch sample of the same instantiation; the CPU
baseline (rank 0, N=1) is the oracle's include/cpp restatement on the host cores.

Before the timed steps a trial picks how frames overlap, with the same grid at every N:
S streams x B frames per shared launch (N = 1) or per RCCL group (N > 1, where the trial
also crosses the interior/edge split and the CUs a shared launch leaves free); the line
reports `frames_in_flight` (S x B) and `frame_latency_ms`. An N > 1 line carries `rccl`
(what RCCL reports about every rank's communicators and devices) and `valid`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_FP32_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 vector (== f32 MFMA) peak
VALU_SIMDS = 1024            # 256 CUs x 4 SIMDs
# how the N = 1 roofline's launch durations are measured (bench.measure)
LAUNCH_TIMING = ("vip_kernel_timing: hipExtLaunchKernel events stamped with each kernel's own begin and end, "
                 "max(4, K/4) frames back to back on one stream after the timed region")
VALU_CYCLES_PER_INSTR = 2    # a wave64 VALU instruction issues over 2 cycles (MI355X_MICROARCH.md)
NBUF = 12


LAUNCH_TIMEOUT_S = 1500.0  # whole N-rank run, launcher included


def free_port() -> int:
    """A TCP port on 127.0.0.1 that was free a moment ago (the rendezvous of the ranks)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_argv(n: int, argv: list, port: int, script: str | None = None) -> list:
    """The child command `python bench.py --gpus N` runs when it is not itself a rank: the
    driver's own form, python -m torch.distributed.run --nnodes=1 --nproc-per-node N
    --master-addr 127.0.0.1 --master-port P bench.py <the same arguments>. torchrun gives
    each rank RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR and MASTER_PORT."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__), *argv]


def launch_ranks(n: int, argv: list, timeout_s: float = LAUNCH_TIMEOUT_S, script: str | None = None) -> int:
    """Run N rank processes (one per GPU) as a child torchrun and return its exit status.

    Called before anything touches the GPU (this process only parsed its arguments), and
    the ranks are children, never an exec of this process. The ranks inherit stdout, so
    rank 0's JSON line is this command's output. Non-zero when any rank fails (torchrun's
    status); 124 when the whole run exceeds timeout_s, after its process group -- the
    launcher and every rank it started -- has been terminated (SIGTERM, then SIGKILL after
    10 s)."""
    return _run_ranks(n, argv, timeout_s, script, capture=False)[0]


def launch_ranks_json(n: int, argv: list, timeout_s: float = LAUNCH_TIMEOUT_S, script: str | None = None):
    """launch_ranks, but the ranks' JSON lines are collected instead of printed (every other
    stdout line is passed through): (exit status, [JSON lines])."""
    return _run_ranks(n, argv, timeout_s, script, capture=True)


def _run_ranks(n, argv, timeout_s, script, capture):
    import signal
    import subprocess
    import threading
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # the host driver supports dmabuf IPC only
    cmd = rank_launch_argv(n, argv, free_port(), script)
    print(f"bench.py: --gpus {n}: starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, env=env, start_new_session=True, stdout=subprocess.PIPE if capture else None,
                            text=True, bufsize=1)
    lines = []
    reader = None
    if capture:
        def pump():
            for line in proc.stdout:
                if line.lstrip().startswith("{"):
                    lines.append(line.strip())
                else:
                    sys.stdout.write(line)
                    sys.stdout.flush()
        reader = threading.Thread(target=pump, daemon=True)
        reader.start()
    try:
        rc = proc.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        print(f"bench.py: the {n}-rank run did not finish in {timeout_s:.0f} s; terminating it", file=sys.stderr,
              flush=True)
        for sig, grace in ((signal.SIGTERM, 10), (signal.SIGKILL, 10)):
            try:
                os.killpg(proc.pid, sig)
            except ProcessLookupError:
                break
            try:
                proc.wait(timeout=grace)
                break
            except subprocess.TimeoutExpired:
                continue
        rc = 124
    if reader is not None:
        reader.join(timeout=10)
    return rc, lines


def align(i: int) -> int:
    """The next step index that starts a whole batch for every B (a multiple of NBUF)."""
    return i + (-i) % NBUF


def halo_batches(streams: int) -> list:
    """Frames per RCCL group the N > 1 native path may use with this many streams: frame i
    runs in batch i // B on stream (i // B) % S, so B * S must divide NBUF for buffer
    i % NBUF to always meet the same stream (its halo receive then stays ordered after its
    last reader)."""
    return [b for b in (1, 2, 3, 4, 6) if NBUF % (b * streams) == 0]


# N > 1 native: frames in flight the trial may use when neither --streams nor the config
# fixes it. A rank's frame is a slab (C2 at N = 8: 270 rows, ~25 us), so a stream's
# exchange latency is about one filter launch; more streams keep the chip fed while the
# halos of the others are in flight (and the small-slab tiling counts them, share = CUs / S).
TRIAL_STREAMS = (2, 3, 4)
# CUs a shared launch (one kernel for a batch's frames, vip_shard_set_frames_launch) leaves to
# the exchange kernels and the other streams' frames. Loopback rehearsal, C2 at 8 GPUs, 3
# frames per group: 0 free 0.0335, 16 free 0.0268 ms per step, against 0.0311 one launch per
# frame (profiles/r04_shared_launch.txt).
SHARED_FREE_CUS = (0, 8, 16, 24, 32)
# N = 1 trial: a form other than the default must be faster by more than this fraction
TRIAL_MARGIN = 0.02


def native_forms(stream_counts, texture: bool, batches=None) -> list:
    """The N > 1 native trial's forms (S streams, split, B frames per RCCL group, shared):
    every S with each B that keeps a buffer on one stream (halo_batches; only `batches` when
    given), the split / one-launch pair (the texture filter has no split), and for B > 1
    after the exchange the B frames in shared launches (vip_shard_set_frames_launch; plain
    and adaptive filters) leaving each of SHARED_FREE_CUS CUs free. shared is None for one
    launch per frame, else that free-CU count. No captured-graph form: graph replay needs
    RCCL >= 2.27.7 and torch binds its own 2.26.6 (vip_shard_set_graph refuses it); it is a
    C/C++ feature (tests/cpp/shard_graph_test)."""
    forms = []
    for n in stream_counts:
        bs = [b for b in halo_batches(n) if batches is None or b in batches]
        for split in ((False,) if texture else (True, False)):
            forms += [(n, split, b, None) for b in bs]
            if not split and not texture:
                forms += [(n, split, b, fc) for b in bs if b > 1 for fc in SHARED_FREE_CUS]
    return forms


def multi_gpu_wall_estimate_s(config: str, n: int, step_ms: float, steps=None, warmup: int = 20,
                              settle_s: float = 6.0) -> float:
    """Worst-case device wall time of one `bench.py --gpus n` line (n > 1, native exchange,
    no --streams / --batch): the settle, every trial form (NBUF untimed + 48 timed steps, plus
    ~5 ms of syncs and barriers each), the warm-up, the K timed steps and the K/4 evented
    steps -- twice for the strong-scaling configs, whose line also measures the weak figure
    (rank startup, imports and RCCL set-up come on top). step_ms: a rank's ms per step in
    that config at that n (the loopback rehearsal lines)."""
    cfg = CONFIGS[config]
    k = DEFAULT_STEPS[config] if steps is None else steps
    forms = native_forms(TRIAL_STREAMS, cfg["kind"] == "texture", cfg.get("native_batches"))
    per = settle_s + len(forms) * ((NBUF + 48) * step_ms * 1e-3 + 5e-3) + (warmup + k + max(4, k // 4)) * step_ms * 1e-3
    strong_with_weak = cfg["kind"] != "texture" and "frame_height" not in cfg
    return per * (2 if strong_with_weak else 1)


def single_gpu_forms(stream_counts, batches=None) -> list:
    """The N = 1 trial's forms for the plain and adaptive filters, the same (S, B) grid as
    the N > 1 trial so both lines are timed in the same forms: S streams of frames in
    flight, B frames per shared launch (vip_*_run_rows_batch; B = 1 one launch per frame)."""
    return [(n, b) for n in stream_counts for b in halo_batches(n) if batches is None or b in batches]


BASELINE_METRIC = "Mpixels/sec bilateral r=7 on 4K RGB; % HBM roofline; 1/2/4/8-GPU scaling"


def circle_taps(r: int) -> int:
    return sum(1 for ky in range(-r, r + 1) for kx in range(-r, r + 1) if kx * kx + ky * ky <= r * r)


CONFIGS = {
    # C1 is the include/cpp (CPU) plumbing case: cpu_baseline times it; the GPU line is
    # the same filter on the same image through the HIP path
    # c1: 4 frames in flight on 4 streams by default (the trial also tries 2 and 3, with B
    # frames per shared launch). The library counts the frames in flight (distinct
    # streams among its recent launches) and picks the throughput tiling by itself: 16-wave
    # 256-pixel tiles, 64 workgroups per 512x512 frame, so four frames run side by side (one
    # frame alone takes 256 4-wave tiles, 10.7 against 14.5 us per launch)
    "c1": dict(kind="bilateral", width=512, frame_height=512, ksize=11, data="lenna", cpu_input="lenna",
               default_streams=4, kernel="void vip::bilateral_kernel<5, 16,",
               kernel_label="bilateral_kernel<R=5> (16 waves x 256-px tiles, 64 per frame, chosen for 4 frames in flight)",
               workload="bilateral r=5 sigma_s=10 sigma_r=30 lenna 512x512"),
    "c2": dict(kind="bilateral", width=3840, rows_per_rank=2160, ksize=15, workload="bilateral r=7 3840x2160 RGB8"),
    "c3": dict(kind="adaptive", width=3840, rows_per_rank=2160, ksize=15,
               workload="adaptive bilateral r=7 3840x2160 RGB8"),
    "c4": dict(kind="texture", width=3840, rows_per_rank=2160, ksize=5, nitr=5,
               workload="bilateral texture k=5 nitr=5 3840x2160 RGB8"),
    # c5 at N = 1: one 805 MB frame per launch (4 rounds of 256 workgroups over 8,192 tiles), so
    # sharing a launch between frames cannot remove a tail worth timing; the N = 1 trial keeps
    # 2 streams and one frame per launch
    # N > 1: one frame per RCCL group (native_batches): a rank's slab is 8192 / 4096 / 2048 rows at
    # N = 2 / 4 / 8, 3-13 ms a step, so shared launches have no tail to remove and the 48-form
    # grid alone would take ~40 s at N = 2 (tests/test_bench_contract.py wall-time bound)
    "c5": dict(kind="bilateral", width=16384, frame_height=16384, ksize=31, single_gpu_forms=[(2, 1)],
               native_batches=[1],
               workload="bilateral r=15 16384x16384 RGB8 row-tiled"),
    # not a BASELINE config: the largest ksize the reference runs (its shared memory
    # fits CUDA's 48 KB default up to 65), on the runtime-radius kernel
    "k65": dict(kind="bilateral", width=3840, rows_per_rank=2160, ksize=65,
                kernel="void vip::stencil_rt_kernel<32, false, true, false>", kernel_label="stencil_rt_kernel (R=32)",
                workload="bilateral r=32 (ksize 65, the largest the reference runs) 3840x2160 RGB8"),
}
# algorithmic FP32 operations per in-support tap: bilateral
# ws*wc (1) + 3 fma (6) + sumk add (1) = 8; adaptive adds the float offset distance:
# 3 subtractions of the offset and the 2 adds of |.|+|.|+|.| = 13 (the integer
# (n - c) differences count no FLOP).
FLOP_PER_TAP = {"bilateral": 8, "adaptive": 13}


DEFAULT_STEPS = {"c1": 6000, "c2": 2000, "c3": 1000, "c4": 500, "c5": 20, "k65": 100}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # defaults: a timed region of ~0.3-0.5 s per config (DEFAULT_STEPS), after a clock
    # settle period and W warm-up steps
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=20)
    # MI355X clocks ramp over ~1 s of sustained load (measured, C2 r=7 4K: 0.219 ms per
    # frame after 3 warm-up steps, 0.179 ms after 200): keep launching untimed steps for
    # this long before the W warm-up steps so the timed steps see the steady clock
    # this long before the W warm-up steps so the timed steps see the steady clock. 6 s, not
    # the 1 s the clocks need: a process-external sampler reading GPU activity every ~5 s
    # (the driver's rocm-smi) then sees the device busy in at least one sample
    p.add_argument("--settle-s", type=float, default=6.0)
    p.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    p.add_argument("--no-cpu-baseline", action="store_true")
    # rehearsal only: gloo + every rank on cuda:0 runs the N>1 code path on a 1-GPU box
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    p.add_argument("--same-device", action="store_true")
    # SURVEY 8(d) inputs: (i) uniform 0..254 like test/random_array.hpp (default), (ii) narrow
    # uniform [100, 120) like sample/benchmark/main.cpp:213, (iii) lenna tiled to the frame
    p.add_argument("--data", default=None, choices=["uniform", "narrow", "lenna"],
                   help="input statistics (default: the config's own -- lenna for c1, uniform otherwise)")
    # the reference's sample/benchmark table instead of the contract line
    p.add_argument("--sample-table", action="store_true")
    p.add_argument("--sample-size", default="100x100")
    # c4 at N=1: two launches per iteration (default, faster) or the guide + JBF fused
    # into one launch (include/vip.h vip_texture_set_mode)
    p.add_argument("--texture-mode", default="two-launch", choices=["two-launch", "fused"])
    # frames in flight: step i runs on HIP stream i % S (one filter handle per stream
    # where the handle owns scratch), so one frame's kernel tails and launch gaps overlap
    # the next frame's start. Measured (scripts/experiments/stream_bench.py, steady clocks): C2
    # 0.178 -> 0.173 ms, C3 0.327 -> 0.323, C4 0.717 -> 0.641 ms per frame with 2; 3 no
    # better. S must divide the 12 rotating buffers (a buffer always meets the same stream)
    p.add_argument("--streams", type=int, default=None, choices=[1, 2, 3, 4, 6],
                   help="fixes S; default: the trial picks 2, 3 or 4 (the config's own first: c1 4, else 2)")
    # N>1: "strong" splits the metric's frame (C2/C3: 3840x2160) over the ranks (default
    # for c2, c3, c5), "weak" gives every rank a 2160-row slab of an (N*2160)-row frame
    # (default for c4). A strong c2/c3 line also carries the weak figure ("weak" key)
    # unless --no-weak.
    p.add_argument("--scaling", default=None, choices=["strong", "weak"])
    p.add_argument("--no-weak", action="store_true")
    # N>1 halo exchange: "native" = include/vip_shard.h (C++ over the library's own RCCL
    # communicator, overlapped with the interior rows; torch.distributed/gloo only for
    # control), "torch" = torch.distributed P2P before the kernel. Default native, torch for
    # the one-GPU gloo rehearsal and the texture filter.
    p.add_argument("--exchange", default=None, choices=["native", "torch"])
    # rehearsal of the N > 1 native path in ONE process (a one-rank RCCL communicator)
    p.add_argument("--rehearse-native", action="store_true")
    # with --rehearse-native: this rank's slab of an N-way row split, whose two row neighbours
    # are the rank itself over a one-rank RCCL communicator (vip_shard_create_loopback), so
    # the real exchange and its trial forms run on one GPU. One rank's slab: not a scaling
    # number.
    p.add_argument("--loopback", type=int, default=0, metavar="N")
    # frames per shared launch (N = 1) / per RCCL group (N > 1): fixes B in the trial
    # (default: the trial picks from halo_batches(S))
    p.add_argument("--batch", type=int, default=None, choices=[1, 2, 3, 4, 6])
    # the plain bilateral kernel's small-frame tiling plans for this many frames in flight
    # (vip_bilateral_set_frames_in_flight) instead of counting the streams in use: a
    # one-stream profiling run of a small frame then launches the instantiation a multi-
    # stream line timed (scripts/gpu.sh iso / pmc)
    p.add_argument("--frames-in-flight", type=int, default=0, choices=[0, 1, 2, 3, 4])
    # --gpus N > 1 without WORLD_SIZE in the environment: this process starts the N ranks
    # itself (a child torchrun) and ends them after this many seconds
    p.add_argument("--launch-timeout", type=float, default=LAUNCH_TIMEOUT_S)
    return p.parse_args()


DATA_DESC = {
    "uniform": "synthetic uniform u8 RGB (torch.randint 0..254)",
    "narrow": "synthetic narrow uniform u8 RGB (torch.randint 100..119, sample/benchmark/main.cpp:213)",
    "lenna": "lenna 512x512 BGR (tests/golden/lenna_bgr.npz) tiled to the frame, row offset per buffer",
}


def make_frames(torch, kind, rows, w, dev, gen, n):
    """n distinct (rows, w, 3) u8 frames resident on dev."""
    if kind == "lenna":
        tile = torch.from_numpy(np.load(os.path.join(ROOT, "tests", "golden", "lenna_bgr.npz"))["bgr"]).to(dev)
        reps = ((rows + 2 * 512 - 1) // 512, (w + 511) // 512, 1)
        big = tile.repeat(*reps)
        # a different vertical phase per buffer so the rotating frames differ
        return [big[(37 * i) % 512:(37 * i) % 512 + rows, :w].contiguous() for i in range(n)]
    lo, hi = (100, 120) if kind == "narrow" else (0, 255)
    return [torch.randint(lo, hi, (rows, w, 3), dtype=torch.uint8, device=dev, generator=gen) for _ in range(n)]


def host_cores() -> tuple[int, str]:
    """Host cores this process may use (affinity set, capped by a cgroup CPU quota
    when one is set) and the CPU model name."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = max(1, min(n, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, model


CPU_SECONDS = 10.0  # CPU work per baseline: at least 10 runs, about this many seconds


def cpu_baseline(cfg) -> dict:
    """include/cpp numerics (oracle CPP profile) on the host cores, row bands in
    parallel threads, on a bounded sample of the same workload: one discarded warm-up,
    then the mean of at least 10 runs (sample/benchmark/main.cpp:20-33, config.toml
    execute_times = 10), as many as fill about CPU_SECONDS. Test infrastructure,
    reported beside the GPU number."""
    from oracle import oracle as o
    threads, model = host_cores()
    w, k = cfg["width"], cfg["ksize"]
    if cfg.get("cpu_input") == "lenna":
        img = np.load(os.path.join(ROOT, "tests", "golden", "lenna_bgr.npz"))["bgr"]
        rows = img.shape[0]
        desc = f"lenna 512x512 (C1), bilateral ksize={k}"
        fn = lambda: o.bilateral(img, k, profile=o.CPP, threads=threads)  # noqa: E731
    elif cfg["kind"] == "texture":
        # every pixel costs the same (no data-dependent work), so independent row bands
        # (each filtered as its own frame) time the same work per pixel
        rows = cfg["rows_per_rank"]  # the whole 4K frame, one row band per thread
        img = o.random_u8(w * rows * 3).reshape(rows, w, 3)
        parts = np.array_split(np.arange(rows), threads)
        desc = f"{w}x{rows} band split in {threads} row bands, texture ksize={k} nitr={cfg['nitr']}"
        fn = lambda: o.bands(lambda a, b: o.texture(img[a:b], k, cfg["nitr"], profile=o.CPP),  # noqa: E731
                             [(int(p[0]), int(p[-1]) + 1) for p in parts], threads)
    else:
        rows = {7: 2160, 15: 256, 32: 64}.get(k // 2, 256)
        img = o.random_u8(w * rows * 3).reshape(rows, w, 3)
        f = o.adaptive if cfg["kind"] == "adaptive" else o.bilateral
        desc = f"{w}x{rows} {'frame' if rows == 2160 else 'band'}, {cfg['kind']} ksize={k}"
        fn = lambda: f(img, k, profile=o.CPP, threads=threads)  # noqa: E731
    fn()  # warm-up, discarded
    ts = []
    while len(ts) < 10 or (sum(ts) < CPU_SECONDS and len(ts) < 2000):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    runs = len(ts)
    dt = sum(ts) / runs
    return dict(value=round(rows * w / dt / 1e6, 4), unit="Mpixels/s", cores=threads, cpu_model=model, runs=runs,
                warmup=1, ms_per_run=round(dt * 1e3, 2), kind="port",
                sample=f"{desc}, {threads} threads, mean of {runs} runs after 1 warm-up (oracle CPP profile = "
                       f"include/cpp numerics, all k*k taps like the reference loop)")


def pmc_summary(config: str, kernel, need: str):
    """(entry, source) from the newest committed rocprofv3 PMC summary of this config
    (profiles/r*_<config>_pmc.json, written by scripts/pmc_summary.py) that holds EXACTLY
    this kernel -- its full template signature, as vip_launched_kernels names the kernel
    the line timed -- with the field `need` ("traffic_bytes", or a counter name); (None,
    None) otherwise. A summary of another instantiation (another tiling, or an older
    build's template list) is stale for this line and is never used."""
    import glob
    if not kernel:
        return None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_pmc.json")), reverse=True):
        with open(f) as fh:
            e = json.load(fh)["kernels"].get(kernel)
        if e and (need in e or need in e.get("counters", {})):
            return e, os.path.relpath(f, ROOT)
    return None, None


def isolated_sample(config: str, kernel) -> dict | None:
    """The committed single-stream launch-duration sample of exactly this kernel: the newest
    profiles/r*_<config>_isolated.csv (scripts/isolated_sample.py over a rocprofv3
    --kernel-trace of `bench.py --streams 1 --batch 1`, one row per launch of the last
    launches of each kernel, none overlapping another) that holds it. The roofline's live
    launch time sits beside it; None when no sample names this instantiation."""
    import csv
    import glob
    import statistics
    if not kernel:
        return None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_isolated.csv")), reverse=True):
        with open(f) as fh:
            rows = [r for r in csv.DictReader(fh) if r["kernel"] == kernel]
        if rows:
            ns = [int(r["duration_ns"]) for r in rows]
            fpl = int(rows[0].get("frames_per_launch") or 1)
            out = dict(source=os.path.relpath(f, ROOT), launches=len(ns), mean_us=round(sum(ns) / len(ns) / 1e3, 2),
                       median_us=round(statistics.median(ns) / 1e3, 2), min_us=round(min(ns) / 1e3, 2),
                       max_us=round(max(ns) / 1e3, 2))
            if fpl > 1:  # a multi-frame kernel profiled with fpl frames per launch
                out.update(frames_per_launch=fpl, mean_us_per_frame=round(sum(ns) / len(ns) / 1e3 / fpl, 3))
            return out
    return None


def pmc_traffic(config: str, kernels: list, per_step: int = 1):
    """HBM bytes per frame of these exact kernels from the committed PMC summaries
    (FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE, scripts/pmc_summary.py; a
    multi-frame kernel's per-dispatch bytes divided by the frames it carried there,
    `frames_per_launch`). Returns (bytes, source) or (None, None) when any kernel has no
    exact summary."""
    total, srcs = 0.0, []
    for k in kernels:
        e, src = pmc_summary(config, k, "traffic_bytes")
        if e is None:
            return None, None
        total += e["traffic_bytes"] / e.get("frames_per_launch", 1)
        srcs.append(src)
    return total * per_step, ", ".join(sorted(set(srcs)))


def launched(kernels: list, prefix: str):
    """The launched kernel (exact name) that starts with prefix, or None; a shared launch's
    multi-frame form of it (`..._frames_kernel<`, vip_*_run_rows_batch) first when present
    (it carries the frames then; a partial last batch of one frame uses the other)."""
    frames = prefix.replace("_kernel<", "_frames_kernel<")
    hit = [k for k in kernels if k.startswith(frames)] + [k for k in kernels if k.startswith(prefix)]
    return hit[0] if hit else None


def valu_issue(config: str, kernel, launch_ms: float):
    """VALU-issue roofline of one kernel: its SQ_INSTS_VALU wave-instructions per frame
    (committed PMC summary of exactly this kernel; a multi-frame kernel's per-dispatch count
    divided by its `frames_per_launch`) / the live event-timed duration per frame, against
    1024 SIMDs issuing one wave64 VALU instruction per 2 cycles (MI355X_MICROARCH.md) at
    the 2.4 GHz maximum clock and at the clock the chip held under this load
    (GRBM_GUI_ACTIVE / 8 XCDs / launch time). None when no summary matches."""
    e, src = pmc_summary(config, kernel, "SQ_INSTS_VALU")
    if e is None:
        return None
    fpl = e.get("frames_per_launch", 1)
    c = {n: v / fpl for n, v in e["counters"].items()}  # per frame
    achieved = c["SQ_INSTS_VALU"] / (launch_ms * 1e-3) / 1e9
    peak = VALU_SIMDS * 2.4 / VALU_CYCLES_PER_INSTR
    out = dict(achieved=round(achieved, 1), peak=round(peak, 1), unit="G wave-instr/s",
               frac=round(achieved / peak, 4), wave_instr_per_launch=c["SQ_INSTS_VALU"], source=src,
               **({"frames_per_launch_profiled": fpl} if fpl > 1 else {}))
    clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / (launch_ms * 1e-3) / 1e9
    # a short launch's GRBM_GUI_ACTIVE also spans its dispatch and drain: a "clock" above
    # the 2.4 GHz maximum is that overhead, not a clock, and is not reported
    if 0 < clk <= 2.4:
        out.update(load_clock_ghz=round(clk, 2), frac_at_load_clock=round(achieved / (VALU_SIMDS * clk / VALU_CYCLES_PER_INSTR), 4))
    if "SQ_LDS_IDX_ACTIVE" in c:  # LDS-array busy: all LDS cycles / (CUs x launch cycles at the load clock)
        out["lds_bank_conflict_cycles"] = c.get("SQ_LDS_BANK_CONFLICT")
        out["lds_array_cycles"] = c["SQ_LDS_IDX_ACTIVE"]
    return out


def texture_roofline(config: str, cfg: dict, px: int, frame_ms: float, stage_ms, kernels: list) -> dict:
    """C4: the dominant kernel of the iteration (the larger of the fused guide stage and
    the joint bilateral, each launch's own duration from vip_kernel_timing) with its own roof, the other one
    beside it, and the pipeline's HBM rate from the bytes the kernels actually move
    (committed PMC summary, per frame) -- not the unfused stage-wise decomposition."""
    nitr, k = cfg["nitr"], cfg["ksize"]
    rj = k - 1                                   # JBF radius: ksize 2k - 1
    taps = circle_taps(rj)
    guide_k = launched(kernels, "void vip::texture_guide_fused_kernel")
    jbf_k = launched(kernels, f"void vip::bilateral_kernel<{rj},")
    out = {"kernels": [guide_k, jbf_k]}
    if stage_ms:
        g_ms, j_ms = stage_ms["guide"], stage_ms["jbf"]
        jbf_tf = 8.0 * taps * px / (j_ms * 1e-3) / 1e12
        jbf = dict(kernel=f"joint bilateral_kernel<R={rj}> (ksize {2 * k - 1}, {taps} taps)", avg_launch_ms=round(j_ms, 4),
                   bound="valu-fp32", achieved=round(jbf_tf, 3), peak=PEAK_FP32_TFLOPS, unit="TFLOP/s",
                   frac=round(jbf_tf / PEAK_FP32_TFLOPS, 4), flop_per_px=8 * taps,
                   valu_issue=valu_issue(config, jbf_k, j_ms), isolated_sample=isolated_sample(config, jbf_k))
        g_gbs = 6.0 * px / (g_ms * 1e-3) / 1e9  # reads the frame, writes the guide
        gtraffic, gsrc = pmc_traffic(config, [guide_k])
        guide = dict(kernel="texture_guide_fused_kernel (gradient + blur/mRTV + argmin/alpha guide, fused)",
                     avg_launch_ms=round(g_ms, 4), bound="valu-issue", bytes_per_px=6,
                     hbm=dict(achieved=round(g_gbs, 2), peak=PEAK_HBM_GBS, unit="GB/s", frac=round(g_gbs / PEAK_HBM_GBS, 4),
                              traffic=gtraffic, traffic_source=gsrc),
                     valu_issue=valu_issue(config, guide_k, g_ms), isolated_sample=isolated_sample(config, guide_k))
        dom, other = (jbf, guide) if j_ms >= g_ms else (guide, jbf)
        if dom is jbf:
            jtraffic, jsrc = pmc_traffic(config, [jbf_k])
            out.update(bound="valu-fp32", achieved=jbf["achieved"], peak=PEAK_FP32_TFLOPS, unit="TFLOP/s",
                       frac=jbf["frac"], traffic=jtraffic, traffic_source=jsrc, traffic_algorithmic=9.0 * px)
        elif guide["valu_issue"]:
            # the guide stage moves 6 B/px (0.1 of HBM): its roof is the VALU issue rate
            # (DESIGN.md section 4), with the HBM figures beside it
            vi = guide["valu_issue"]
            out.update(bound="valu-issue", achieved=vi["achieved"], peak=vi["peak"], unit=vi["unit"], frac=vi["frac"],
                       hbm=guide["hbm"], traffic=guide["hbm"]["traffic"],
                       traffic_source=guide["hbm"]["traffic_source"], traffic_algorithmic=6.0 * px)
        else:
            out.update(bound="hbm", achieved=guide["hbm"]["achieved"], peak=PEAK_HBM_GBS, unit="GB/s",
                       frac=guide["hbm"]["frac"], traffic=guide["hbm"]["traffic"], traffic_source=guide["hbm"]["traffic_source"],
                       traffic_algorithmic=6.0 * px)
        out.update(kernel=dom["kernel"], avg_launch_ms=dom["avg_launch_ms"], dominant=dom, other=other,
                   launch_timing=LAUNCH_TIMING)
    traffic, tsrc = pmc_traffic(config, [guide_k, jbf_k], nitr)
    pipe = dict(frame_ms=round(frame_ms, 4), launches=2 * nitr, traffic_per_frame=traffic, traffic_source=tsrc)
    if traffic:
        gbs = traffic / (frame_ms * 1e-3) / 1e9
        pipe.update(hbm_achieved=round(gbs, 2), hbm_peak=PEAK_HBM_GBS, hbm_frac=round(gbs / PEAK_HBM_GBS, 4),
                    fused_floor_bytes=6.0 * px * nitr)
    out["pipeline"] = pipe
    return out


def texture_fused_roofline(cfg: dict, px: int, frame_ms: float, kernels: list) -> dict:
    """C4 in FUSED mode: one launch per iteration (texture_iteration_fused_kernel), so the
    kernel is the whole iteration: FP32 rate of its JBF taps (8 FLOP per in-disc tap, the
    guide stage's work beside it uncounted), VALU issue and HBM traffic from the
    committed PMC summary of this mode (profiles/r*_c4fused_pmc.json)."""
    nitr, k = cfg["nitr"], cfg["ksize"]
    taps = circle_taps(k - 1)
    launch_ms = frame_ms / nitr
    kern = launched(kernels, "void vip::texture_iteration_fused_kernel")
    tf = 8.0 * taps * px / (launch_ms * 1e-3) / 1e12
    traffic, tsrc = pmc_traffic("c4fused", [kern])
    return dict(kernel=f"texture_iteration_fused_kernel (guide + JBF ksize {2 * k - 1} in one launch)", kernel_name=kern,
                avg_launch_ms=round(launch_ms, 4), bound="valu-fp32", achieved=round(tf, 3), peak=PEAK_FP32_TFLOPS,
                unit="TFLOP/s", frac=round(tf / PEAK_FP32_TFLOPS, 4), traffic=traffic, traffic_source=tsrc,
                traffic_algorithmic=6.0 * px, valu_issue=valu_issue("c4fused", kern, launch_ms),
                pipeline=dict(frame_ms=round(frame_ms, 4), launches=nitr,
                              traffic_per_frame=traffic * nitr if traffic else None,
                              fused_floor_bytes=6.0 * px * nitr))


def sample_table(args) -> None:
    """The reference's sample/benchmark/main.cpp:105-213 table: every filter timed on the
    include/cpp path and on the GPU path side by side, on a randu(100, 120) image of
    --sample-size (default 100x100), ksize 9, texture ksize 9 nitr 3
    (sample/benchmark/config.toml), one discarded warm-up then the mean of 10 calls
    (MEASURE, :20-33). cpp = the oracle's CPP profile (include/cpp numerics) in row bands
    on the host cores; hip = the blocking public API on device-resident frames."""
    import torch

    import various_image_processings_amd as vip
    from oracle import oracle as o
    w, h = (int(v) for v in args.sample_size.split("x"))
    threads, model = host_cores()
    img = 100 + o.random_u8(w * h * 3, 20).reshape(h, w, 3)
    d_src = torch.from_numpy(img).cuda()
    d_dst, d_mag = torch.empty_like(d_src), torch.empty((h, w), dtype=torch.float32, device="cuda")
    bf, abf = vip.CudaBilateralFilter(w, h, 9), vip.CudaAdaptiveBilateralFilter(w, h, 9)
    tf = vip.CudaBilateralTextureFilter(w, h, 9, 3)

    def grad_hip():
        vip.cuda_gradient(d_src, d_mag, w, h, 3)
        torch.cuda.synchronize()  # the reference's call returns unsynchronised; its D2H syncs

    rows = [
        ("gradient", lambda: o.gradient(img, o.CPP), grad_hip),
        ("bilateral filter", lambda: o.bilateral(img, 9, profile=o.CPP, threads=threads),
         lambda: bf.bilateral_filter(d_src, d_dst)),
        ("adaptive bilateral filter", lambda: o.adaptive(img, 9, profile=o.CPP, threads=threads),
         lambda: abf.execute(d_src, d_dst)),
        ("bilateral texture filter", lambda: o.texture(img, 9, 3, o.CPP), lambda: tf.execute(d_src, d_dst)),
    ]

    def measure(fn, n=10):
        fn()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        return (time.perf_counter() - t0) / n * 1e3

    print(f"Parameters\n\twidth {w} height {h} execute times 10 ksize 9 texture ksize 9 nitr 3 "
          f"(cpp: {threads} threads, {model})\n")
    for name, cpp, hip in rows:
        print(f"{name + ' [cpp]':40s} : {measure(cpp):10.6f} [msec]")
        print(f"{name + ' [hip]':40s} : {measure(hip):10.6f} [msec]")


def init_distributed(args, rank, dev):
    """Process group for N>1. With the native exchange (include/vip_shard.h) the halos
    move over the library's own RCCL communicator and torch.distributed only carries the
    control traffic (the communicator id, barriers, the max over ranks): gloo. Otherwise
    the halos move through torch.distributed P2P: nccl (= RCCL), or gloo for the one-GPU
    rehearsal. A rank that cannot join ends the run with a message and status 3, never a
    hang: bounded rendezvous and collective timeouts."""
    import datetime

    import torch.distributed as dist
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    backend = "gloo" if args.exchange == "native" else args.backend
    try:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=180))
        else:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=180))
        dist.barrier()  # communicator up before the first halo exchange
    except Exception as e:  # noqa: BLE001
        print(f"bench.py rank {rank}: process group ({backend}) failed: {e!r}", file=sys.stderr, flush=True)
        os._exit(3)
    return backend


def native_shards(args, cfg, frame_h, rank, world, n):
    """This rank's n NativeShards, one per stream, each over its own RCCL communicator
    (vip_shard_create / vip_shard_create_texture with a communicator id from rank 0): a
    stream's exchanges then never share a communicator or a communication stream with the
    other stream's, and a texture shard's scratch slabs serve one frame at a time. Returns
    (shards, None), or (None, reason) when any rank failed -- all ranks agree (gloo)."""
    import torch
    import torch.distributed as dist

    from various_image_processings_amd.sharded import NativeShard, native_unique_id
    shards, err = [], ""
    for _ in range(n):
        box = [native_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        ns = None
        if not err:
            try:
                lb = args.loopback > 1  # rehearsal: the middle rank of an N-way split, itself as neighbours
                ns = NativeShard(cfg["width"], frame_h, cfg["ksize"], args.loopback // 2 if lb else rank,
                                 args.loopback if lb else world, box[0],
                                 adaptive=cfg["kind"] == "adaptive", timeout_ms=120000,
                                 nitr=cfg["nitr"] if cfg["kind"] == "texture" else None, loopback=lb)
            except Exception as e:  # noqa: BLE001
                err = f"rank {rank}: {e}"
                print(f"bench.py {err}", file=sys.stderr, flush=True)
        ok = torch.tensor([0 if ns is None else 1], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok[0]) == 0:
            return None, err or "another rank failed to create its shard"
        shards.append(ns)
    return shards, None


def device_identity(torch, dev) -> str:
    """This rank's device as the PCI location torch reports (domain:bus:device), else its
    uuid, else its index: what tells two ranks' devices apart without an RCCL readback."""
    p = torch.cuda.get_device_properties(dev)
    if all(hasattr(p, a) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id")):
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    return str(getattr(p, "uuid", None) or f"index {torch.cuda.current_device()}")


def rccl_evidence(shards, rank, world, expected_count) -> dict:
    """What RCCL itself reports about the communicators this run exchanged over: every
    rank's ncclCommCount / ncclCommUserRank / ncclCommCuDevice (vip_shard_comm_info, for each
    of its shards, one per stream) and its device's PCI bus id, gathered to every rank over
    the control process group. `problems` lists what would make an N-GPU line not an N-GPU
    measurement: a communicator of another size, a rank that is not its own user rank, or
    two ranks on one device."""
    import torch.distributed as dist

    from various_image_processings_amd.sharded import rccl_version
    try:
        infos = [s.comm_info() for s in shards]
        mine = dict(rank=rank, count=infos[0]["count"], user_rank=infos[0]["user_rank"], device=infos[0]["device"],
                    pci_bus_id=infos[0]["pci_bus_id"], shards=len(infos),
                    shards_agree=all((i["count"], i["user_rank"], i["device"]) ==
                                     (infos[0]["count"], infos[0]["user_rank"], infos[0]["device"]) for i in infos))
    except Exception as e:  # every rank still reaches the gather (a raise here would hang the peers)
        mine = dict(rank=rank, count=None, user_rank=None, device=None, pci_bus_id=f"unknown (rank {rank})",
                    shards=len(shards), shards_agree=False, error=repr(e))
    ranks = [None] * world
    if world > 1:
        dist.all_gather_object(ranks, mine)
    else:
        ranks = [mine]
    counts = sorted({r_["count"] for r_ in ranks}, key=lambda c: (c is None, c or 0))
    buses = [r_["pci_bus_id"] for r_ in ranks]
    problems = [f"rank {r_['rank']}: comm_info failed: {r_['error']}" for r_ in ranks if r_.get("error")]
    if counts != [expected_count]:
        problems.append(f"communicator sizes {counts}, expected {expected_count}")
    if expected_count > 1 and any(r_["user_rank"] != r_["rank"] for r_ in ranks):
        problems.append("a rank's RCCL user rank differs from its process rank")
    if not all(r_["shards_agree"] for r_ in ranks):
        problems.append("a rank's communicators (one per stream) disagree")
    if len(set(buses)) != len(buses):
        problems.append(f"{len(buses)} ranks on {len(set(buses))} distinct devices")
    return dict(ranks=ranks, count=counts[0] if len(counts) == 1 else counts, distinct_devices=len(set(buses)),
                rccl_version=rccl_version(),
                problems=problems)


def measure(args, cfg, frame_h, torch, dev, rank, world, streams, state, s_forms=None):
    """Build one workload (buffers, handles) and time it: W warm-up steps, then K steps
    between barriers + device syncs, max over ranks. Returns the measured quantities.
    s_forms: the stream counts the trial may pick from (at most len(streams)); default: all
    the streams."""
    import torch.distributed as dist

    from various_image_processings_amd.filters import _TextureImpl, launched_kernels
    from various_image_processings_amd.sharded import ShardedBilateral, ShardedTexture, exchange_halo

    launched_kernels()  # clear this thread's launch log: the workload below names its kernels

    S = len(streams)
    stream = streams[0]
    sraw = [st.cuda_stream for st in streams]  # hipStream_t of each stream
    w, k = cfg["width"], cfg["ksize"]
    gen = torch.Generator(device=dev)
    gen.manual_seed(42 + rank)
    res = dict(frame_h=frame_h, exchange=None, stage_ms=None, samples=None)
    native = False
    single_batch = False  # N = 1 plain / adaptive: the trial may share launches between frames
    cdev = dev if state.get("backend") == "nccl" else "cpu"  # control tensors of the process group
    multi = state.get("multi", world > 1)  # a process group is up (N > 1, or --rehearse-native)

    if cfg["kind"] == "texture" and world == 1 and not args.loopback:
        rows = frame_h
        geo = None
        # one handle per stream: a texture handle owns its ping-pong and guide frames
        texs = [_TextureImpl(w, rows, k, cfg["nitr"]) for _ in range(S)]
        if args.texture_mode == "fused":
            for t_ in texs:
                t_.set_mode(_TextureImpl.FUSED)
        srcs = make_frames(torch, args.data, rows, w, dev, gen, NBUF)
        dsts = [torch.empty((rows, w, 3), dtype=torch.uint8, device=dev) for _ in range(NBUF)]
        sp, dp = [t.data_ptr() for t in srcs], [t.data_ptr() for t in dsts]

        def run(i, s=stream, h=0):  # s is streams[h]; raw addresses keep host work per launch small
            texs[h].execute(sp[i % NBUF], dp[i % NBUF], stream=sraw[h])
    else:
        shards = None
        if multi and args.exchange == "native":
            # one shard (own RCCL communicator, own communication stream) per stream
            shards, why = native_shards(args, cfg, frame_h, rank, world, S)
            if shards is None:  # fall back to torch.distributed P2P over a new RCCL group
                if "torch_group" not in state:
                    state["torch_group"] = dist.new_group(backend="nccl" if args.backend == "nccl" else "gloo")
                res["exchange_fallback"] = why
        native = shards is not None
        if native:
            sb = shards[0]
            # RCCL's own account of the communicators (checked into the line's "valid")
            res["rccl"] = rccl_evidence(shards, rank, world, 1 if args.loopback > 1 else world)
        elif cfg["kind"] == "texture":
            # torch P2P: one halo exchange of nitr * texture_halo_rows(k) rows per frame,
            # then shrinking ghost zones (sharded.ShardedTexture; one per stream: it owns
            # scratch slabs)
            sts = [ShardedTexture(w, frame_h, k, cfg["nitr"], rank, world) for _ in range(S)]
            sb = sts[0]
        else:
            # the handle holds only read-only LUTs: one serves every stream
            sb = ShardedBilateral(w, frame_h, k, rank, world, adaptive=cfg["kind"] == "adaptive")
        geo = sb.geo
        rows = geo.own
        srcs = make_frames(torch, args.data, geo.slab_rows, w, dev, gen, NBUF)
        dsts = [torch.empty((rows, w, 3), dtype=torch.uint8, device=dev) for _ in range(NBUF)]
        sp, dp = [t.data_ptr() for t in srcs], [t.data_ptr() for t in dsts]
        if native:
            nruns = [x.launcher() for x in shards]  # vip_shard_run with its arguments bound
            # vip_shard_run_batch: several frames' halos in one RCCL group
            nbatches = [x.batch_launcher() for x in shards]

            def run(i, s=stream, h=0):  # exchange + filter (vip_shard_run) on stream h's shard
                nruns[h](sp[i % NBUF], dp[i % NBUF], sraw[h])
        elif cfg["kind"] == "texture":
            def run(i, s=stream, h=0):
                sts[h].filter(srcs[i % NBUF], dsts[i % NBUF], stream=s, exchange=False)
        else:
            launch = sb.launcher()  # the C entry point with its arguments bound

            def run(i, s=stream, h=0):  # s is streams[h]; raw addresses keep host work per launch small
                launch(sp[i % NBUF], dp[i % NBUF], sraw[h])
            if not multi:
                # N = 1: B frames in one shared launch (vip_*_run_rows_batch, all CUs), the
                # form the N > 1 line may pick after its exchange
                single_batch = True
                nbatches = [sb.batch_launcher()] * len(streams)
    has_peers = world > 1 or (native and args.loopback > 1)
    res["exchange"] = (None if not multi else
                       ("native vip_shard (RCCL ncclSend/ncclRecv with the row neighbours; one communicator per "
                        "stream)" if has_peers else "native vip_shard, one rank: no neighbours, no exchange")
                       if native else
                       f"torch.distributed P2P ({state.get('backend', args.backend)}), serial before the kernel")

    # N=1: the kernels run back to back and ev0..ev1 / steps is the kernel time per frame
    # (with S > 1 streams: per frame with S frames in flight).
    # N>1: the timed steps carry no inner events (an event between launches costs stream
    # time); max(4, K/4) further steps after the timed region, on one stream, carry them:
    # torch exchange -- before the exchange, between exchange and kernel, after it;
    # native -- vip_shard_run_timed's run start, halos in, interior done, edges done.
    marks = []
    group = state.get("torch_group")
    # frames may share one RCCL group (N > 1 native, vip_shard_run_batch; the group's cost is
    # mostly fixed, profiles/r03_rccl_enqueue.txt) or one launch (N = 1, vip_*_run_rows_batch)
    # per B frames. Frame i then runs on stream (i // B) % S; B * S divides NBUF, so buffer
    # i % NBUF still always meets the same stream and a halo receive into it stays ordered
    # after its last reader.
    batching = native or single_batch
    s_forms = list(s_forms or [S])
    hb = dict(B=1, S=s_forms[0], pending=[])  # S: the streams in use (the trial may change it)

    def flush():
        if hb["pending"]:
            h = (hb["pending"][0] // hb["B"]) % hb["S"]
            nbatches[h]([sp[j % NBUF] for j in hb["pending"]], [dp[j % NBUF] for j in hb["pending"]], sraw[h])
            hb["pending"].clear()

    def step(i, sample=False):
        # step i on stream i % S; buffer i % NBUF therefore always meets the same stream
        # (S divides NBUF), so a halo receive into it is ordered after its last reader
        h = 0 if sample else i % hb["S"]
        s = streams[h]
        if batching and not sample and hb["B"] > 1:
            # batches end on multiples of B (a phase end flushes a partial one), so every
            # frame of a batch has the same i // B, hence the same stream
            hb["pending"].append(i)
            if (i + 1) % hb["B"] == 0:
                flush()
            return
        if batching and sample:
            flush()
        if not multi and not sample:  # one GPU: the launch names its stream; no torch stream context
            run(i, s, h)
            return
        if native:
            if sample:
                m = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                with torch.cuda.stream(s):
                    sb.filter_timed(srcs[i % NBUF], dsts[i % NBUF], m, stream=s)
                marks.append(m)
            else:
                run(i, s, h)
            return
        with torch.cuda.stream(s):  # RCCL orders its P2P against the current stream
            if sample:
                m = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                m[0].record(s)
            if world > 1:
                exchange_halo(srcs[i % NBUF], geo, group)
            if sample:
                m[1].record(s)
            run(i, s, h)
            if sample:
                m[2].record(s)
                marks.append(m)

    # clock settle (untimed): steps for --settle-s seconds of wall time, checked every
    # few steps with a device sync; then the W warm-up steps. At N>1 every step exchanges
    # (the ranks must issue the same P2P sequence), so the settle runs a step count
    # agreed by rank 0.
    t_settle, i_settle = time.perf_counter(), 0
    if not multi:
        # one stream: back-to-back launches warm the clocks as well as overlapped ones, and a
        # kernel trace of the run (rocprofv3, the driver's own profile) then shows launch
        # durations rather than spans of launches sharing the chip
        while time.perf_counter() - t_settle < args.settle_s:
            for _ in range(8):
                run(i_settle, streams[0], 0)
                i_settle += 1
            torch.cuda.synchronize(dev)
    else:
        for _ in range(8):
            step(i_settle)
            i_settle += 1
        torch.cuda.synchronize(dev)
        per = max(1e-4, (time.perf_counter() - t_settle) / 8)
        n = torch.tensor([int(args.settle_s / per)], dtype=torch.int64, device=cdev)
        dist.broadcast(n, src=0)
        for _ in range(int(n[0])):
            step(i_settle)
            i_settle += 1
        torch.cuda.synchronize(dev)
    # every phase below starts on a multiple of NBUF (= 12, a multiple of every B), so its
    # batches are whole: frames per RCCL group / per shared launch are always B (skipped
    # indices run nothing; buffer i % NBUF keeps its stream)
    i_settle = align(i_settle)
    batches = None if args.batch is None else [args.batch]
    native_batches = batches if batches is not None else cfg.get("native_batches")
    if native and not has_peers:
        # one rank (--rehearse-native): no halo moves, so split / batch forms would only
        # time noise between identical launches; keep the defaults and say so
        res["split"] = dict(chosen="one launch (no neighbours: no exchange, no trial)", trial_ms_per_step={})
        res["split_on"] = False
    elif native:
        # vip_shard_set_split: interior rows under the exchange then the two edge bands,
        # or one launch after the exchange (fewer launches; with two frames in flight the
        # exchange still overlaps the other frame's kernel); and B frames per RCCL group.
        # Which is faster depends on the exchange's latency and host cost on this machine:
        # time each (max over ranks) and keep the fastest. The texture filter has no split
        # (every iteration reads the halo region).
        # With several stream counts (TRIAL_STREAMS), S is a trial dimension too: frames in
        # flight hide one stream's exchange latency behind the others' launches.
        trial = {}
        n_trial = 48  # a multiple of every B
        forms = native_forms(s_forms, cfg["kind"] == "texture", native_batches)
        if not forms:
            raise SystemExit(f"bench.py: --batch {args.batch} fits none of the stream counts {s_forms}")
        for n_s, split, b, shared in forms:
            for x in shards:
                x.set_split(split)
                x.set_frames_launch(shared is not None, shared or 0)
            hb["B"], hb["S"] = b, n_s
            for _ in range(NBUF):  # untimed: every (buffer, stream) pair once in this form
                step(i_settle)
                i_settle += 1
            flush()
            torch.cuda.synchronize(dev)
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(n_trial):
                step(i_settle)
                i_settle += 1
            flush()
            torch.cuda.synchronize(dev)
            dist.barrier()
            dt = torch.tensor([(time.perf_counter() - t0) / n_trial * 1e3], dtype=torch.float64, device=cdev)
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            trial[(n_s, split, b, shared)] = float(dt[0])
        best_s, best_split, best_b, best_shared = min(trial, key=trial.get)
        res["split_on"] = best_split
        for x in shards:
            x.set_split(best_split)
            x.set_frames_launch(best_shared is not None, best_shared or 0)
        hb["B"], hb["S"] = best_b, best_s
        res["streams"] = best_s
        res["exchange"] += ("; interior rows overlapped with the exchange, then the edge bands" if best_split
                            else "; one launch over the own rows after the exchange")
        if best_b > 1:
            res["exchange"] += f"; the halos of {best_b} frames per RCCL group"
            if best_shared is not None:
                res["exchange"] += ", filtered in one launch" + (f" leaving {best_shared} CUs free" if best_shared else "")
        res["split"] = dict(chosen="interior rows during the exchange, then the edge bands" if best_split
                            else "one launch after the exchange",
                            frames_launch=best_shared,
                            trial_ms_per_step={(f"s{s_}_" if len(s_forms) > 1 else "")
                                               + ("split" if sp_ else "one_launch") + (f"_batch{b_}" if b_ > 1 else "")
                                               + ("" if sh_ is None else "_one_kernel" + (f"_free{sh_}" if sh_ else "")):
                                               round(v, 4)
                                               for (s_, sp_, b_, sh_), v in trial.items()})
        res["halo_batch"] = best_b
    elif single_batch or (not multi and len(s_forms) > 1):
        # N = 1, the same (S, B) grid as the N > 1 trial: S frames in flight, B frames per
        # shared launch (the texture filter: S only, one handle per stream). Each form runs
        # as many steps as fill about a quarter of the timed region (a multiple of every B)
        # after one untimed pass over the buffers; keep the fastest.
        trial = {}
        n_trial = NBUF * max(4, args.steps // 48)
        s_first = sorted(s_forms, key=lambda n: n != args.streams)  # the config's stream count first
        forms = [f for f in cfg.get("single_gpu_forms", single_gpu_forms(s_first, batches))
                 if f[0] <= len(streams) and (batches is None or f[1] in batches)] or single_gpu_forms(s_first, batches)
        if not single_batch:  # no shared launches: one frame per launch on each stream count
            forms = [(n, 1) for n in s_first]
        if not forms:
            raise SystemExit(f"bench.py: --batch {args.batch} fits none of the stream counts {s_forms}")
        for n_s, b in forms:
            hb["B"], hb["S"] = b, n_s
            for _ in range(NBUF):
                step(i_settle)
                i_settle += 1
            flush()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(n_trial):
                step(i_settle)
                i_settle += 1
            flush()
            torch.cuda.synchronize(dev)
            trial[(n_s, b)] = (time.perf_counter() - t0) / n_trial * 1e3
        best_s, best_b = min(trial, key=trial.get)
        # trial noise is ~1 % at C2 (r05 lines: s2_batch1 0.1679 against s2_batch2 0.1678 ms;
        # on another box 0.1717-0.1743 over forms that do the same work): another form replaces
        # the default (the first form: one frame per launch on the config's streams, whose
        # kernel the committed PMC and launch samples hold) only when it is faster by more
        # than TRIAL_MARGIN (C1's shared launches win by 17-20 %)
        default = forms[0]
        if trial[(best_s, best_b)] * (1 + TRIAL_MARGIN) >= trial[default]:
            best_s, best_b = default
        hb["B"], hb["S"] = best_b, best_s
        res["streams"] = best_s
        res["batch"] = dict(chosen=best_b, streams=best_s, default=f"s{default[0]}_batch{default[1]}",
                            margin=TRIAL_MARGIN, trial_steps=n_trial,
                            trial_ms_per_step={f"s{s_}_batch{b_}": round(v, 4) for (s_, b_), v in trial.items()})
    res["settle_steps"] = i_settle
    S_run = hb["S"]  # streams the timed steps use
    base = i_settle
    for i in range(args.warmup):
        step(base + i)
    t_first = align(base + args.warmup)  # the first timed step
    if batching:
        flush()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    launched_kernels()  # the line names the kernels of the timed steps (not of the settle's first launches)
    t0 = time.perf_counter()
    ev0.record(stream)
    for s in streams[1:S_run]:
        s.wait_event(ev0)
    for i in range(args.steps):
        step(t_first + i)
    if batching:
        flush()  # a partial last batch is part of the timed frames
    host_s = time.perf_counter() - t0  # every step enqueued
    res["kernels_timed"] = launched_kernels()
    for s in streams[1:S_run]:
        stream.wait_stream(s)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    after = align(t_first + args.steps)
    single_ms = None
    parts = None
    B = hb["B"]
    res["frames_in_flight"] = S_run * B
    if multi:
        for i in range(max(4, args.steps // 4)):
            step(after + i, sample=True)
        torch.cuda.synchronize(dev)
        avg = lambda a, b: sum(m[a].elapsed_time(m[b]) for m in marks) / len(marks)  # noqa: E731
        if native:
            # vip_shard_run_timed: events[2] after the interior rows (split) or once the
            # halos are in on the filter stream (one launch)
            if res.get("split_on"):
                parts = dict(exchange_ms=avg(0, 1), interior_ms=avg(0, 2), edges_ms=avg(2, 3), run_ms=avg(0, 3))
            else:
                parts = dict(exchange_ms=avg(0, 1), wait_ms=avg(0, 2), filter_ms=avg(2, 3), run_ms=avg(0, 3))
            kernel_ms = parts["run_ms"]
            if B > 1 and has_peers:
                # one frame's latency in the chosen form: a whole group of B frames (one RCCL
                # group, then its launches) alone on one stream, from the point its own rows
                # are written to the last output row -- what the last frame of a group waits
                lat = []
                j0 = after + max(4, args.steps // 4)
                j0 += (-j0) % B
                for g_ in range(max(2, args.steps // (4 * B))):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    nbatches[0]([sp[(j0 + g_ * B + f) % NBUF] for f in range(B)],
                                [dp[(j0 + g_ * B + f) % NBUF] for f in range(B)], sraw[0])
                    e1.record(stream)
                    lat.append((e0, e1))
                torch.cuda.synchronize(dev)
                parts["group_latency_ms"] = sum(a.elapsed_time(b) for a, b in lat) / len(lat)
        else:
            parts = dict(exchange_ms=avg(0, 1), kernel_ms=avg(1, 2))
            kernel_ms = parts["kernel_ms"]
    else:
        kernel_ms = ev0.elapsed_time(ev1) / args.steps
        # The roofline is per kernel: its launch durations come from max(4, K/4) more frames
        # (a multiple of B) on ONE stream, back to back, after the timed region, each launch
        # carrying events the runtime stamps with the kernel's own begin and end
        # (vip_kernel_timing, hipExtLaunchKernel: no marker packet in the stream, so these
        # are the durations rocprofv3 --kernel-trace reports). The S-stream launches of the
        # timed region overlap each other, so their spans are not kernel durations; with
        # B > 1 one launch carries B frames and the duration is divided by B.
        import various_image_processings_amd as vip_
        n1 = max(4, args.steps // 4)
        n1 += (-n1) % B
        timed_kernels = set(res["kernels_timed"])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        per_frame = 2 * cfg["nitr"] if cfg["kind"] == "texture" else 1

        def one_stream(first):
            with vip_.kernel_timing(n1 * per_frame) as kt:
                e0.record(stream)
                if B > 1:
                    for j in range(first, first + n1, B):
                        nbatches[0]([sp[(j + f) % NBUF] for f in range(B)], [dp[(j + f) % NBUF] for f in range(B)],
                                    sraw[0])
                else:
                    for i in range(n1):
                        run(first + i)
                e1.record(stream)
            torch.cuda.synchronize(dev)
            return e0.elapsed_time(e1) / n1, kt.durations()

        single_ms, kdur = one_stream(after + (-after) % B)
        if not set(launched_kernels()) <= timed_kernels:
            # one stream made the library pick another tiling than the frames in flight
            # did (its small-frame tiling counts the streams in use): time the timed
            # region's kernel, back to back on one stream, with the frame count forced
            # to the S the timed frames had (vip_bilateral_set_frames_in_flight)
            vip_.set_bilateral_frames_in_flight(min(S_run, 4))
            try:
                single_ms, kdur = one_stream(after + n1 + (-(after + n1)) % B)
            finally:  # back to the run's own setting (--frames-in-flight, else counted)
                vip_.set_bilateral_frames_in_flight(args.frames_in_flight)
            res["launch_timing"] = (f"one stream, the tiling planned for the timed region's {S_run} frames in "
                                    f"flight (vip_bilateral_set_frames_in_flight)")
            if not set(launched_kernels()) <= timed_kernels:
                res["launch_timing"] += "; WARNING: another kernel ran"
        if B > 1:
            res["launch_timing"] = (res.get("launch_timing", "one stream") +
                                    f"; {B} frames per launch, duration per frame")
        # per kernel: launches, mean / min / max duration (ms, per launch)
        res["kernel_durations"] = {n: dict(launches=len(v), mean_ms=sum(v) / len(v), min_ms=min(v), max_ms=max(v))
                                   for n, v in kdur.items()}
        res["span_one_stream_ms"] = single_ms  # per frame, launch gaps included
    launch_ms = single_ms if single_ms is not None else kernel_ms
    # one frame's latency: the whole launch that carries it on an idle stream (N = 1) or
    # its RCCL group's exchange and launches (N > 1); the reference's public call blocks for
    # one frame (sample/benchmark/main.cpp:20-33 times one call per frame)
    if not multi:
        res["frame_latency_ms"] = launch_ms * B
    elif parts:
        res["frame_latency_ms"] = parts.get("group_latency_ms", parts.get("run_ms", kernel_ms))
    fused = cfg["kind"] == "texture" and world == 1 and not args.loopback and args.texture_mode == "fused"
    if cfg["kind"] == "texture" and world == 1 and not args.loopback and not fused:
        # per-stage kernel durations (vip_kernel_timing), per launch
        kd = res["kernel_durations"]
        g_ = [v["mean_ms"] for n, v in kd.items() if n.startswith("void vip::texture_guide_fused_kernel")]
        j_ = [v["mean_ms"] for n, v in kd.items() if n.startswith(f"void vip::bilateral_kernel<{k - 1},")]
        if g_ and j_:
            res["stage_ms"] = {"guide": g_[0], "jbf": j_[0]}
    keys = ["elapsed", "launch", "host", "latency"] + (sorted(parts) if parts else [])
    vals = [elapsed, launch_ms, host_s, res.get("frame_latency_ms", 0.0)] + \
        ([parts[x] for x in sorted(parts)] if parts else [])
    t = torch.tensor(vals, dtype=torch.float64, device=cdev)
    if multi:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    got = dict(zip(keys, (float(v) for v in t)))
    if "frame_latency_ms" in res:
        res["frame_latency_ms"] = got["latency"]
    # every kernel instantiation this workload launched (N = 1 with S > 1 streams: those of the
    # timed frames)
    res["kernels"] = res.pop("kernels_timed")
    launched_kernels()
    if native:  # release the communicators on every rank at the same point (not at GC time)
        torch.cuda.synchronize(dev)
        dist.barrier()
        for x in shards:
            x.close()
    res.update(elapsed=got["elapsed"], launch_ms=got["launch"], host_s=got["host"], frame_ms=kernel_ms, rows=rows, geo=geo,
               parts={x: got[x] for x in sorted(parts)} if parts else None, native=native, fused=fused, batch=B,
               **({"batch_trial": res["batch"]} if isinstance(res.get("batch"), dict) else {}))
    return res


def main():
    args = parse()
    if args.sample_table:
        sample_table(args)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.rehearse_native:
        # plain `python bench.py --gpus N`: start the N ranks (nothing has touched the GPU)
        # one run, one HIP runtime and one RCCL per rank (torch's): no graph form, no retry
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout))
    import torch
    import torch.distributed as dist

    cfg = CONFIGS[args.config]
    if args.steps is None:
        args.steps = DEFAULT_STEPS[args.config]
    if args.data is None:  # the config's own input unless one is asked for
        args.data = cfg.get("data", "uniform")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} rank(s)", file=sys.stderr,
              flush=True)
    if args.same_device:
        local = 0
    if args.exchange is None:
        # the native RCCL exchange needs one GPU per rank; the one-GPU rehearsal (gloo,
        # every rank on cuda:0) keeps the torch P2P path
        args.exchange = "torch" if (args.same_device or args.backend == "gloo") else "native"
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    state = {"multi": world > 1 or args.rehearse_native}
    if args.rehearse_native:
        # one rank through the N > 1 native path (a one-rank RCCL communicator, no
        # neighbours): id broadcast, vip_shard_create, the split timing, the evented steps
        if world != 1:
            raise SystemExit("--rehearse-native is a single-process run")
        args.exchange = "native"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29400 + os.getpid() % 500))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if state["multi"]:
        state["backend"] = init_distributed(args, rank, dev)

    import various_image_processings_amd as vip  # noqa: F401  (loads libvip_hip.so or raises)

    if args.frames_in_flight:
        vip.set_bilateral_frames_in_flight(args.frames_in_flight)
    fixed_streams = args.streams
    S = args.streams = fixed_streams or cfg.get("default_streams", 2)
    if "tiling" in cfg and world == 1:  # the config's tile shape (include/vip.h tuning knobs)
        vip.set_bilateral_waves(cfg["tiling"][0])
        vip.set_bilateral_wide(cfg["tiling"][1])
    # stream 0 is torch's current stream (S = 1 is exactly the single-stream bench); with
    # a process group every stream is a created one (graph capture needs a non-null stream)
    streams = ([torch.cuda.Stream(dev) for _ in range(S)] if state["multi"] else
               [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)])
    if args.scaling is None:
        # the metric's frame (3840x2160; C5 16384^2) split over the ranks; the texture
        # filter's 45-row ghost halo makes a split 4K frame mostly redundant work, so C4
        # scales weakly (a 2160-row slab per rank)
        args.scaling = "weak" if cfg["kind"] == "texture" else "strong"
    if "frame_height" in cfg:
        args.scaling = "strong"
    per_rank = cfg.get("rows_per_rank")
    if args.loopback and not args.rehearse_native:
        raise SystemExit("--loopback N is a --rehearse-native option")
    gw = args.loopback if args.loopback > 1 else world  # ranks of the row split (geometry)
    sharded = gw > 1  # this process filters a slab of a larger frame
    frame_h = cfg.get("frame_height") or (per_rank * gw if args.scaling == "weak" else per_rank)
    s_forms = None
    if not fixed_streams and ((sharded and args.exchange == "native") or
                              (not state["multi"] and (cfg["kind"] in FLOP_PER_TAP or
                                                       (cfg["kind"] == "texture" and args.texture_mode != "fused")))):
        # the trial also picks the frames in flight (TRIAL_STREAMS): at N > 1 native one
        # shard per stream; at N = 1 (plain and adaptive filters) the same S x B grid, so
        # the N = 1 and N > 1 lines are timed in the same forms
        s_forms = list(TRIAL_STREAMS)
        streams += [torch.cuda.Stream(dev) for _ in range(max(s_forms) - len(streams))]
    m = measure(args, cfg, frame_h, torch, dev, rank, world, streams, state, s_forms)
    weak = None
    if world > 1 and args.scaling == "strong" and per_rank and not args.no_weak:
        # the weak-scaling figure beside it: a full 2160-row slab per rank of an
        # (N*2160)x3840 frame
        wm = measure(args, cfg, per_rank * world, torch, dev, rank, world, streams, state, s_forms)
        wpx = wm["rows"] * cfg["width"] * world
        weak = dict(value=round(wpx / (wm["elapsed"] / args.steps) / 1e6, 2),
                    ms_per_step=round(wm["elapsed"] / args.steps * 1e3, 4), frame=f"{cfg['width']}x{per_rank * world}",
                    rows_per_rank=wm["rows"], **({k_: round(v, 4) for k_, v in wm["parts"].items()} if wm["parts"] else {}))

    w, k = cfg["width"], cfg["ksize"]
    r = k // 2
    elapsed, launch_ms, rows, geo = m["elapsed"], m["launch_ms"], m["rows"], m["geo"]
    px_per_rank = rows * w
    # the whole frame's pixels (every rank's); a loopback rehearsal processes one slab only
    total_px = px_per_rank if args.loopback > 1 else frame_h * w
    ms_per_step = elapsed / args.steps * 1e3
    value = total_px / (elapsed / args.steps) / 1e6

    if m["fused"]:
        roof = texture_fused_roofline(cfg, px_per_rank, launch_ms, m["kernels"])
    elif cfg["kind"] == "texture":
        roof = texture_roofline(args.config, cfg, px_per_rank, launch_ms, m["stage_ms"], m["kernels"])
    else:
        taps = circle_taps(r)
        flops = FLOP_PER_TAP[cfg["kind"]] * taps * px_per_rank
        # the exact instantiation this run launched (vip_launched_kernels), for the PMC lookup
        kname = launched(m["kernels"], cfg.get("kernel", f"void vip::{cfg['kind']}_kernel<{r},"))
        # a shared launch (vip_*_run_rows_batch, B > 1) carries B frames: durations, PMC
        # counts and bytes are per frame (the summaries record the frames per dispatch
        # they were profiled with)
        fpl = m["batch"] if kname and "_frames_kernel<" in kname else 1
        # N = 1: the kernel's own begin-to-end duration per frame (vip_kernel_timing); N > 1:
        # the per-rank device time of one step (exchange included, below)
        kd = (m.get("kernel_durations") or {}).get(kname)
        dur_ms = kd["mean_ms"] / fpl if kd else launch_ms
        tflops = flops / (dur_ms * 1e-3) / 1e12
        hbm = 6.0 * px_per_rank / (dur_ms * 1e-3) / 1e9
        traffic, tsrc = (None, None) if sharded else pmc_traffic(args.config, [kname])
        roof = dict(bound="valu-fp32", achieved=round(tflops, 3), peak=PEAK_FP32_TFLOPS, unit="TFLOP/s",
                    frac=round(tflops / PEAK_FP32_TFLOPS, 4), traffic=traffic, traffic_source=tsrc,
                    traffic_algorithmic=6.0 * px_per_rank,
                    kernel=cfg.get("kernel_label", f"{cfg['kind']}_kernel<R={r}>"), kernel_name=kname,
                    avg_launch_ms=round(dur_ms, 4),
                    **({"launch_timing": LAUNCH_TIMING, "launches_timed": kd["launches"],
                        "span_one_stream_ms": round(m["span_one_stream_ms"], 4)} if kd else {}),
                    flop_per_px=FLOP_PER_TAP[cfg["kind"]] * taps, in_support_taps=taps,
                    gtaps_per_s=round(taps * px_per_rank / (dur_ms * 1e-3) / 1e9, 1),
                    hbm=dict(achieved=round(hbm, 2), peak=PEAK_HBM_GBS, unit="GB/s", frac=round(hbm / PEAK_HBM_GBS, 5),
                             bytes_per_px=6))
        if not sharded:  # the committed PMC summaries are whole-frame launches
            roof["valu_issue"] = valu_issue(args.config, kname, dur_ms)
            if fpl > 1:
                roof["frames_per_launch"] = fpl
            roof["isolated_sample"] = isolated_sample(args.config, kname)
            if m["frames_in_flight"] > 1:  # the chip's rate with frames in flight (launches overlap)
                fl = flops / (ms_per_step * 1e-3) / 1e12
                roof["in_flight"] = dict(achieved=round(fl, 3), frac=round(fl / PEAK_FP32_TFLOPS, 4), unit="TFLOP/s",
                                         note=f"{m['frames_in_flight']} frames in flight: flops per frame / ms_per_step")
        else:
            roof["avg_launch_note"] = ("per-rank device time of one step on one stream: "
                                       + ("vip_shard_run (exchange, then the own rows: "
                                          + m["split"]["chosen"] + ")" if m["native"]
                                          else "the kernel after the serial exchange"))

    parts = m["parts"] or {}
    out = {
        "metric": BASELINE_METRIC if args.config == "c2" else f"Mpixels/sec {cfg['workload']}",
        "value": round(value, 2),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        # host time to enqueue the K timed steps (max over ranks), per step: below
        # ms_per_step, the host keeps ahead of the GPU
        "host_ms_per_step": round(m["host_s"] / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": DATA_DESC[args.data] + ", resident in HBM; f32 weights/sums",
        "config": {"workload": cfg["workload"], "ksize": k, "sigma_space": 10.0, "sigma_color": 30.0,
                   "frame": f"{w}x{frame_h}", "rows_per_rank": rows, "data": args.data,
                   "parallelism": f"row-tiled x{gw}" + (f" + {geo.radius}-row halo sendrecv" if sharded and geo else ""),
                   **({"tiling": cfg["kernel_label"]} if "tiling" in cfg and world == 1 else {}),
                   **({"texture_mode": args.texture_mode} if cfg["kind"] == "texture" and world == 1 else {}),
                   **({"backend": state.get("backend"), "exchange": m["exchange"]} if state["multi"] else {}),
                   **({"exchange_fallback": m["exchange_fallback"]} if m.get("exchange_fallback") else {})},
        "roofline": roof,
        "kernels": m["kernels"],
        # per step, max over ranks: one frame on one stream (N>1: with its exchange),
        # event-timed in max(4, K/4) steps after the timed region; the roofline's launch
        # durations come from it
        "kernel_ms": round(launch_ms, 4),
        # frames in flight on S streams (step i on stream i % S); at N=1 and S>1 the
        # timed region's device time per frame, all streams together
        "streams": m.get("streams", S),
        # S streams x B frames per shared launch (N = 1) or per RCCL group (N > 1)
        "frames_in_flight": m["frames_in_flight"],
        **({"frame_latency_ms": round(m["frame_latency_ms"], 4)} if m.get("frame_latency_ms") else {}),
        **({"frame_ms_in_flight": round(m["frame_ms"], 4)} if world == 1 and m["frames_in_flight"] > 1 else {}),
        "settle": {"seconds": args.settle_s, "steps": m["settle_steps"]},
        **{k_: round(v, 4) for k_, v in parts.items()},
        **({"split": m["split"]} if m.get("split") else {}),
        **({"launch_timing": m["launch_timing"]} if m.get("launch_timing") else {}),
        **({"halo_batch": m["halo_batch"]} if m.get("halo_batch") else {}),
        **({"batch": m["batch_trial"]} if m.get("batch_trial") else {}),
        **({"weak": weak} if weak else {}),
    }
    bt = m.get("batch_trial")
    if world == 1 and bt and bt.get("chosen", 1) > 1:
        # a shared-launch form won the N = 1 trial (C1): the value is a batched throughput;
        # the reference times one blocking call per frame (sample/benchmark/main.cpp:20-33),
        # so the default form's own rate (one frame per launch, the trial's time) sits beside it
        d_ms = bt["trial_ms_per_step"][bt["default"]]
        out["throughput_form"] = (f"batched throughput: {bt['streams']} streams x {bt['chosen']} frames per shared "
                                  f"launch ({m['frames_in_flight']} frames in flight)")
        out["one_frame_per_launch"] = dict(form=bt["default"], ms_per_step=round(d_ms, 4),
                                           value=round(total_px / (d_ms * 1e-3) / 1e6, 2),
                                           source="the N = 1 trial's time of the default form")
    if state["multi"]:
        # an N-GPU line must show that RCCL saw N ranks on N distinct devices
        problems = []
        if m.get("rccl"):
            out["rccl"] = m["rccl"]
            problems += m["rccl"]["problems"]
        elif args.exchange == "native":
            problems.append("no RCCL communicator to report (no native shard)")
        if m.get("exchange_fallback"):
            problems.append(f"exchange fell back to torch.distributed P2P: {m['exchange_fallback']}")
        if not m.get("rccl") and world > 1:
            # torch P2P exchange (or a fallback): no RCCL readback, but the ranks' devices
            # must still be distinct (the --same-device gloo rehearsal is not an N-GPU run)
            ids = [None] * world
            dist.all_gather_object(ids, device_identity(torch, dev))
            out["devices"] = ids
            if len(set(ids)) != world:
                problems.append(f"{world} ranks on {len(set(ids))} distinct devices")
        if world != args.gpus:
            problems.append(f"--gpus {args.gpus} but {world} rank(s) ran")
        out["valid"] = not problems
        if problems:
            out["invalid_reason"] = "; ".join(problems)
    from various_image_processings_amd import build_info
    out["build"] = build_info.check()  # the loaded libraries against the sources beside them
    if args.loopback > 1:
        out["rehearsal"] = (f"one GPU: the middle rank's slab of a {args.loopback}-way row split, its two neighbours "
                            f"the rank itself over a one-rank RCCL communicator (vip_shard_create_loopback); value "
                            f"counts this slab only -- not a scaling number")
    if rank == 0 and not sharded and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(cfg)
        except Exception as e:  # the baseline is reported, never required
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if state["multi"]:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
