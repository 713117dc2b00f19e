"""Row-tile sharding of one frame across GPUs with an r-row halo exchange.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, over
xGMI). Rank i owns frame rows [row_begin, row_end) in a slab buffer laid out as

    rows [0, r)                 halo above   (received from rank i-1)
    rows [r, r + n)             own rows
    rows [r + n, 2r + n)        halo below   (received from rank i+1)

exchange() sends the own top/bottom r rows to the neighbours and receives their
edge rows into the halos: one sendrecv pair per neighbour, no collective. The
filter then runs on the slab with neighbour rows clamped to the rows that are
valid: at the frame's first/last rank the halo is absent and clamping to the
own rows reproduces the reference's replicate border exactly
(src/bilateral_filter_impl.cu:50-51), so sharded output == single-GPU output.

The reference has no multi-device code; this is the
north_star's row-tiled C5 configuration. ShardedTexture extends it to the
iterated texture filter with one wide halo per frame.
"""
from __future__ import annotations

from dataclasses import dataclass


def shard_rows(frame_height: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced row ranges (first ranks take the remainder)."""
    base, rem = divmod(frame_height, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


@dataclass
class SlabGeometry:
    width: int
    frame_height: int
    radius: int
    rank: int
    world: int

    def __post_init__(self):
        # Checked identically on every rank, before any P2P call: the thinnest shard
        # (shard_rows gives sizes that differ by one) must still cover a full halo,
        # or the ranks whose shards are thick enough would block in the exchange
        # while the others raise.
        if not (0 <= self.rank < self.world):
            raise ValueError(f"rank {self.rank} outside world {self.world}")
        if self.world > 1 and self.radius > 0 and self.frame_height // self.world < self.radius:
            raise ValueError(f"{self.frame_height} rows over {self.world} ranks: the thinnest shard "
                             f"({self.frame_height // self.world} rows) is thinner than the {self.radius}-row halo")

    @property
    def rows(self) -> tuple[int, int]:
        return shard_rows(self.frame_height, self.world, self.rank)

    @property
    def own(self) -> int:
        b, e = self.rows
        return e - b

    @property
    def slab_rows(self) -> int:
        return self.own + 2 * self.radius

    @property
    def has_above(self) -> bool:
        return self.rank > 0

    @property
    def has_below(self) -> bool:
        return self.rank < self.world - 1

    def clamp_range(self) -> tuple[int, int]:
        """Slab rows the filter may read (neighbour rows clamp into this range)."""
        r = self.radius
        lo = 0 if self.has_above else r
        hi = self.slab_rows if self.has_below else r + self.own
        return lo, hi


def split_bands(geo: SlabGeometry) -> tuple[tuple[int, int], list[tuple[int, int]]]:
    """Own rows split for overlapping the exchange (== vip_shard.hip interior/edges):
    the interior (row0, rows) = (r, own - 2r) reads only own rows, so it can run while
    the halos move; the two edge bands [(0, r), (own - r, r)] need the halos. Thin shards
    (own <= 2r) have no interior and edge bands that tile the own rows."""
    r, own = geo.radius, geo.own
    top = min(r, own)
    b0 = max(own - r, top)
    return (r, max(0, own - 2 * r)), [(0, top), (b0, own - b0)]


def exchange_halo(slab, geo: SlabGeometry, group=None) -> None:
    """Fill slab's halo rows from the neighbouring ranks (blocking).

    `slab` is a (slab_rows, width, C) contiguous tensor on this rank's device;
    for the gloo backend a CPU tensor. Uses batched point-to-point ops so both
    directions and both neighbours are in flight together.
    """
    import torch.distributed as dist

    r, n = geo.radius, geo.own
    if geo.world == 1 or r == 0:
        return
    # gloo moves host tensors only: a device slab is staged through host copies
    # (CPU rehearsal of the N>1 path; with nccl = RCCL the slab rows go GPU to GPU)
    staged = slab.is_cuda and dist.get_backend(group) == "gloo"
    if not staged:
        # the per-step host work is only the batched launch: the row views and P2P
        # ops of a slab buffer are built once (bench.py rotates a fixed set of slabs)
        key = (slab.data_ptr(), tuple(slab.shape), slab.device, group)
        cache = geo.__dict__.setdefault("_p2p_ops", {})
        ops = cache.get(key)
        if ops is None:
            ops = []
            if geo.has_above:
                ops.append(dist.P2POp(dist.isend, slab[r:2 * r], geo.rank - 1, group))
                ops.append(dist.P2POp(dist.irecv, slab[0:r], geo.rank - 1, group))
            if geo.has_below:
                ops.append(dist.P2POp(dist.isend, slab[n:n + r], geo.rank + 1, group))
                ops.append(dist.P2POp(dist.irecv, slab[n + r:n + 2 * r], geo.rank + 1, group))
            if len(cache) >= 32:  # the views keep their slabs alive: bound the cache
                cache.pop(next(iter(cache)))
            cache[key] = ops
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        return
    sends, recvs = [], []
    if geo.has_above:
        sends.append((slab[r:2 * r], geo.rank - 1))
        recvs.append((slab[0:r], geo.rank - 1))
    if geo.has_below:
        sends.append((slab[n:n + r], geo.rank + 1))
        recvs.append((slab[n + r:n + 2 * r], geo.rank + 1))
    if staged:
        sends = [(t.cpu(), p) for t, p in sends]
        bufs = [(t, t.cpu(), p) for t, p in recvs]
        recvs = [(h, p) for _, h, p in bufs]
    ops = [dist.P2POp(dist.isend, t, p, group) for t, p in sends] + \
          [dist.P2POp(dist.irecv, t, p, group) for t, p in recvs]
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    if staged:
        for dst, host, _ in bufs:
            dst.copy_(host)


def _exchange_on(slab, geo: SlabGeometry, stream) -> None:
    """exchange_halo ordered before later work on `stream`.

    With RCCL, a request's wait() orders the received rows only before torch's
    CURRENT stream; the kernel that reads them runs on `stream` (a torch.cuda.Stream,
    a raw hipStream_t address, or None = the current stream), so the exchange runs
    with `stream` made current.
    """
    if stream is None:
        exchange_halo(slab, geo)
        return
    import torch
    s = stream if isinstance(stream, torch.cuda.Stream) else torch.cuda.ExternalStream(int(stream), device=slab.device)
    with torch.cuda.stream(s):
        exchange_halo(slab, geo)


class ShardedBilateral:
    """Bilateral (or adaptive) filter of a row-sharded frame on the HIP kernels."""

    def __init__(self, width: int, frame_height: int, ksize: int, rank: int, world: int, sigma_space: float = 10.0,
                 sigma_color: float = 30.0, adaptive: bool = False, numerics: int = 0):
        from .filters import _AdaptiveImpl, _BilateralImpl
        self.geo = SlabGeometry(width, frame_height, ksize // 2, rank, world)
        cls = _AdaptiveImpl if adaptive else _BilateralImpl
        # the handle's height only sizes nothing on the row-band path; use the slab
        self.impl = cls(width, self.geo.slab_rows, ksize, sigma_space, sigma_color, numerics)
        self.adaptive = adaptive
        self._clamp = self.geo.clamp_range()

    def filter(self, slab, out, stream=None, exchange: bool = True, split: bool = False) -> None:
        """slab: (own + 2r, W, 3) uint8 with own rows filled; out: (own, W, 3).
        exchange and split: the interior rows first (they read no halo), then the halo
        exchange, then the two edge bands (split_bands) -- the kernel's work that can
        proceed while the halos move is queued ahead of the exchange. Default: the
        exchange, then one launch (the edge launches cost more than a small exchange
        hides; vip_shard_set_split)."""
        g = self.geo
        if exchange and split and g.world > 1:
            (i0, ni), edges = split_bands(g)
            if ni > 0:
                self._rows(slab, out, i0, ni, stream)
                _exchange_on(slab, g, stream)
                for e0, ne in edges:
                    self._rows(slab, out, e0, ne, stream)
                return
        if exchange:
            _exchange_on(slab, g, stream)
        self._rows(slab, out, 0, g.own, stream)

    def _rows(self, slab, out, row0: int, rows: int, stream) -> None:
        """Own rows [row0, row0 + rows) of the slab -> the same rows of out."""
        if rows <= 0:
            return
        lo, hi = self._clamp
        o = out + row0 * self.geo.width * 3 if isinstance(out, int) else out[row0:row0 + rows]
        self.impl.run_rows(slab, o, rows, self.geo.radius + row0, lo, hi, stream=stream)

    def launcher(self):
        """A lean callable f(slab_ptr, out_ptr, hip_stream) for the whole own-row range
        (no exchange): the C entry point with every other argument bound, so that a
        small frame's host cost per launch is the ctypes call alone. Raw device addresses,
        unchecked (the benchmark's own preallocated buffers)."""
        from . import _lib
        g = self.geo
        lo, hi = self._clamp
        p = g.width * 3
        fn = getattr(_lib.lib(), "vip_adaptive_run_rows" if self.adaptive else "vip_bilateral_run_rows")
        h = self.impl._h
        name = fn.__name__
        if self.adaptive:
            def run(src, dst, stream):
                rc = fn(h, src, p, dst, p, g.own, g.radius, lo, hi, stream)
                if rc:
                    _lib.check(name, rc)
        else:
            def run(src, dst, stream):
                rc = fn(h, src, p, None, 0, dst, p, g.own, g.radius, lo, hi, stream)
                if rc:
                    _lib.check(name, rc)
        return run

    def batch_launcher(self, free_cus: int = 0):
        """A lean callable f(src_ptrs, dst_ptrs, hip_stream): the whole own-row range of
        several frames in shared launches (vip_bilateral_run_rows_batch /
        vip_adaptive_run_rows_batch, up to 6 frames per launch), no exchange. Raw device
        addresses, unchecked."""
        import ctypes
        from . import _lib
        g = self.geo
        lo, hi = self._clamp
        p = g.width * 3
        name = "vip_adaptive_run_rows_batch" if self.adaptive else "vip_bilateral_run_rows_batch"
        fn = getattr(_lib.lib(), name)
        h = self.impl._h

        def run(srcs, dsts, stream):
            n = len(srcs)
            rc = fn(h, n, (ctypes.c_void_p * n)(*srcs), p, (ctypes.c_void_p * n)(*dsts), p, g.own, g.radius, lo, hi,
                    int(free_cus), stream)
            if rc:
                _lib.check(name, rc)
        return run


def texture_halo_rows(ksize: int) -> int:
    """Rows one texture iteration reaches beyond its output rows: the JBF radius
    k-1 on the guide plus the guide's reach (gradient 1 + blur/mRTV k/2 + argmin k/2)
    into the image; == include/vip.h vip_texture_halo_rows."""
    return (ksize - 1) + 2 * (ksize // 2) + 1


class ShardedTexture:
    """Bilateral texture filter of a row-sharded frame.

    The halo is exchanged ONCE per frame, nitr * texture_halo_rows(k) rows deep
    (45 rows for k=5, nitr=5), instead of once per iteration: iteration t then
    computes the own rows plus a margin of (nitr-1-t) * halo rows on each side
    (ghost-zone shrinking), so the last iteration's own rows are exact. The
    redundant margin work is 2 * halo * (nitr-1) * nitr / 2 row-iterations per
    frame (about 1.7 % at 2160 own rows, k=5, nitr=5); one exchange replaces nitr.
    """

    def __init__(self, width: int, frame_height: int, ksize: int, nitr: int, rank: int, world: int,
                 numerics: int = 0):
        from .filters import _TextureImpl
        self.step = texture_halo_rows(ksize)
        self.nitr = nitr
        self.geo = SlabGeometry(width, frame_height, self.step * nitr if world > 1 else 0, rank, world)
        self.impl = _TextureImpl(width, self.geo.slab_rows, ksize, nitr, numerics)
        self._scratch = None

    def filter(self, slab, out, stream=None, exchange: bool = True) -> None:
        """slab: (own + 2 * halo, W, 3) uint8 with own rows filled; out: (own, W, 3)."""
        import torch
        g = self.geo
        if exchange:
            _exchange_on(slab, g, stream)
        if self.nitr == 0:
            out.copy_(slab[g.radius:g.radius + g.own])
            return
        if self._scratch is None or self._scratch[0].shape != slab.shape or self._scratch[0].device != slab.device:
            self._scratch = (torch.empty_like(slab), torch.empty_like(slab))
        lo, hi = g.clamp_range()
        a = slab
        for t in range(self.nitr):
            m = (self.nitr - 1 - t) * self.step
            r0, r1 = max(lo, g.radius - m), min(hi, g.radius + g.own + m)
            if t == self.nitr - 1:
                self.impl.iterate_rows(a, out, g.radius, g.own, lo, hi, stream=stream)
            else:
                b = self._scratch[t % 2]
                self.impl.iterate_rows(a, b[r0:r1], r0, r1 - r0, lo, hi, stream=stream)
                a = b


# ---------------------------------------------------------------------------
# Native path: include/vip_shard.h (libvip_shard.so). The exchange runs in C++ over the
# library's own RCCL communicator (ncclSend/ncclRecv with the row neighbours), enqueued
# on a communication stream together with the interior rows on the filter stream; the
# two r-row edge bands follow once the halos are in. Same SlabGeometry, same results.
# ---------------------------------------------------------------------------
def _shard_kind(adaptive: bool) -> int:
    from . import _lib
    return _lib.VIP_FILTER_ADAPTIVE if adaptive else _lib.VIP_FILTER_BILATERAL


def native_unique_id() -> bytes:
    """The communicator id (ncclGetUniqueId) rank 0 creates and broadcasts."""
    import ctypes
    from . import _shard_lib as S
    buf = ctypes.create_string_buffer(S.VIP_SHARD_ID_BYTES)
    S.call("vip_shard_unique_id", buf)
    return buf.raw


def native_rows(frame_height: int, world: int, rank: int) -> tuple[int, int]:
    """vip_shard_rows: (first row, own rows), == shard_rows (no device call)."""
    import ctypes
    from . import _shard_lib as S
    b, n = ctypes.c_int(), ctypes.c_int()
    S.call("vip_shard_rows", frame_height, world, rank, ctypes.byref(b), ctypes.byref(n))
    return b.value, b.value + n.value


def rccl_version() -> int:
    """ncclGetVersion of the RCCL bound in this process (vip_shard_rccl_version)."""
    import ctypes
    from . import _shard_lib as S
    v = ctypes.c_int()
    S.call("vip_shard_rccl_version", ctypes.byref(v))
    return v.value


def _native_halo(ksize: int, nitr) -> int:
    """Halo rows of a native shard: r = ksize / 2, or nitr texture iterations deep."""
    return ksize // 2 if nitr is None else nitr * texture_halo_rows(ksize)


class NativeShard:
    """This rank's shard of a row-sharded frame (one process per GPU, RCCL transport).
    nitr given: the bilateral texture filter (vip_shard_create_texture; ksize is its k).
    loopback=True (unique_id ignored): vip_shard_create_loopback, the test transport whose
    row neighbours are this shard itself over a one-rank communicator (one GPU)."""

    def __init__(self, width: int, frame_height: int, ksize: int, rank: int, world: int, unique_id: bytes,
                 sigma_space: float = 10.0, sigma_color: float = 30.0, adaptive: bool = False, numerics: int = 0,
                 timeout_ms: int = 180000, nitr=None, loopback: bool = False):
        import ctypes
        from . import _lib
        from . import _shard_lib as S
        self._h = ctypes.c_void_p()
        if loopback:
            kind = _lib.VIP_FILTER_TEXTURE if nitr is not None else _shard_kind(adaptive)
            S.call("vip_shard_create_loopback", ctypes.byref(self._h), kind, width, frame_height, ksize, sigma_space,
                   sigma_color, nitr or 0, numerics, world, rank, int(timeout_ms))
            self.geo = SlabGeometry(width, frame_height, _native_halo(ksize, nitr), rank, world)
            return
        idb = ctypes.create_string_buffer(bytes(unique_id or b""), S.VIP_SHARD_ID_BYTES)
        if nitr is None:
            S.call("vip_shard_create", ctypes.byref(self._h), _shard_kind(adaptive), width, frame_height, ksize,
                   sigma_space, sigma_color, numerics, world, rank, idb, int(timeout_ms))
        else:
            S.call("vip_shard_create_texture", ctypes.byref(self._h), width, frame_height, ksize, nitr, numerics,
                   world, rank, idb, int(timeout_ms))
        self.geo = SlabGeometry(width, frame_height, _native_halo(ksize, nitr), rank, world)

    def set_split(self, split: bool) -> None:
        """vip_shard_set_split: interior rows during the exchange, then the edge bands
        (True), or one launch after the exchange (False, the default)."""
        from . import _shard_lib as S
        S.call("vip_shard_set_split", self._h, 1 if split else 0)

    def set_graph(self, on: bool) -> None:
        """vip_shard_set_graph: replay one captured hipGraph per (slab, out, stream). Raises
        ShardError (VIP_ERR_UNSUPPORTED) when the RCCL bound in this process is older than
        2.27.7 -- inside a torch process that is torch's bundled 2.26.6, so graph mode is a
        C/C++ feature (tests/cpp/shard_graph_test)."""
        from . import _shard_lib as S
        S.call("vip_shard_set_graph", self._h, 1 if on else 0)

    def comm_info(self) -> dict:
        """What RCCL reports about this shard's communicator (vip_shard_comm_info:
        ncclCommCount, ncclCommUserRank, ncclCommCuDevice) and the device's PCI bus id."""
        import ctypes
        from . import _shard_lib as S
        c, r, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        S.call("vip_shard_comm_info", self._h, ctypes.byref(c), ctypes.byref(r), ctypes.byref(d))
        bus = ctypes.create_string_buffer(32)
        S.call("vip_shard_pci_bus_id", self._h, bus, 32)
        return dict(count=c.value, user_rank=r.value, device=d.value, pci_bus_id=bus.value.decode())

    def set_frames_launch(self, on: bool, free_cus: int = 0) -> None:
        """vip_shard_set_frames_launch: a batch's frames share filter launches that leave
        free_cus CUs to concurrent work (True) or launch one by one (False, the default)."""
        from . import _shard_lib as S
        S.call("vip_shard_set_frames_launch", self._h, 1 if on else 0, int(free_cus))

    def graph_count(self) -> int:
        import ctypes
        from . import _shard_lib as S
        n = ctypes.c_int()
        S.call("vip_shard_graph_count", self._h, ctypes.byref(n))
        return n.value

    def filter(self, slab, out, stream=None) -> None:
        """slab: (own + 2r, W, 3) uint8 with own rows filled; out: (own, W, 3). Asynchronous."""
        from . import _shard_lib as S
        from .filters import _ptr, _stream
        p = self.geo.width * 3
        S.call("vip_shard_run", self._h, _ptr(slab, p * self.geo.slab_rows), _ptr(out, p * self.geo.own), p,
               _stream(stream))

    def launcher(self):
        """A lean callable f(slab_ptr, out_ptr, hip_stream) for vip_shard_run with the
        handle and pitch bound (raw device addresses, unchecked): the host cost per frame
        is the ctypes call, which matters when a rank's slab takes ~25 us on the GPU."""
        from . import _shard_lib as S
        fn = S.lib().vip_shard_run
        h, p = self._h, self.geo.width * 3

        def run(slab, out, stream):
            rc = fn(h, slab, out, p, stream)
            if rc:
                raise S.ShardError("vip_shard_run", rc)
        return run

    def batch_launcher(self):
        """A lean callable f(slab_ptrs, out_ptrs, hip_stream) for vip_shard_run_batch: the
        halos of all the frames in one RCCL group, then their launches (raw device
        addresses, unchecked). Every rank must batch the same frames."""
        import ctypes
        from . import _shard_lib as S
        fn = S.lib().vip_shard_run_batch
        h, p = self._h, self.geo.width * 3

        def run(slabs, outs, stream):
            n = len(slabs)
            rc = fn(h, n, (ctypes.c_void_p * n)(*slabs), (ctypes.c_void_p * n)(*outs), p, stream)
            if rc:
                raise S.ShardError("vip_shard_run_batch", rc)
        return run

    def filter_timed(self, slab, out, events, stream=None) -> None:
        """events: 4 timing-enabled torch.cuda.Event (vip_shard_run_timed): run start,
        halos received (communication stream), interior done, edges done."""
        import ctypes
        from . import _shard_lib as S
        from .filters import _ptr, _stream
        for e in events:
            e.record()  # materialise the hipEvent_t behind the torch event
        arr = (ctypes.c_void_p * 4)(*[e.cuda_event for e in events])
        p = self.geo.width * 3
        S.call("vip_shard_run_timed", self._h, _ptr(slab, p * self.geo.slab_rows), _ptr(out, p * self.geo.own), p,
               _stream(stream), arr)

    def close(self) -> None:
        """vip_shard_destroy now (releases the communicator: call it at the same point on
        every rank rather than leaving it to the garbage collector)."""
        if self._h and self._h.value:
            from . import _shard_lib as S
            S.lib().vip_shard_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardGroup:
    """All shards of a frame in ONE process: transport LOCAL (every slab on the current
    device, halos by device copies -- the native exchange path on one GPU) or RCCL over
    `devices` (one communicator per device, ncclCommInitAll's pattern)."""

    def __init__(self, n: int, width: int, frame_height: int, ksize: int, transport: int = 1, devices=None,
                 sigma_space: float = 10.0, sigma_color: float = 30.0, adaptive: bool = False, numerics: int = 0,
                 timeout_ms: int = 180000, nitr=None):
        import ctypes
        from . import _shard_lib as S
        self.n = n
        self._hs = (ctypes.c_void_p * n)()
        devs = None if devices is None else (ctypes.c_int * n)(*devices)
        if nitr is None:
            S.call("vip_shard_create_group", self._hs, n, transport, devs, _shard_kind(adaptive), width, frame_height,
                   ksize, sigma_space, sigma_color, numerics, int(timeout_ms))
        else:
            S.call("vip_shard_create_group_texture", self._hs, n, transport, devs, width, frame_height, ksize, nitr,
                   numerics, int(timeout_ms))
        self.geos = [SlabGeometry(width, frame_height, _native_halo(ksize, nitr), i, n) for i in range(n)]

    def set_split(self, split: bool) -> None:
        from . import _shard_lib as S
        for i in range(self.n):
            S.call("vip_shard_set_split", self._hs[i], 1 if split else 0)

    def filter(self, slabs, outs, streams) -> None:
        import ctypes
        from . import _shard_lib as S
        from .filters import _ptr, _stream
        n = self.n
        g = self.geos
        p = g[0].width * 3
        sl = (ctypes.c_void_p * n)(*[_ptr(s, p * g[i].slab_rows) for i, s in enumerate(slabs)])
        ou = (ctypes.c_void_p * n)(*[_ptr(o, p * g[i].own) for i, o in enumerate(outs)])
        st = (ctypes.c_void_p * n)(*[_stream(s) for s in streams])
        S.call("vip_shard_run_group", self._hs, n, sl, ou, p, st)

    def __del__(self):
        try:
            from . import _shard_lib as S
            for i in range(self.n):
                if self._hs[i]:
                    S.lib().vip_shard_destroy(self._hs[i])
                    self._hs[i] = None
        except Exception:
            pass
