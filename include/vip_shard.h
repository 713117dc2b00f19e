/*
 * vip_shard.h -- row-sharded frames over several GPUs with an RCCL halo exchange
 * (C ABI, libvip_shard.so; links libvip_hip.so and RCCL).
 *
 * No reference counterpart: yuyuyu-bot/various_image_processings has no multi-device
 * code. This is the north_star's row-tiled configuration (BASELINE
 * config 5: bilateral r=15 on 16384x16384 over 8 GPUs, "2r-row halo exchanged via RCCL
 * sendrecv over xGMI") as a native entry point for C/C++ callers, who would otherwise have
 * to write their own exchange around vip_bilateral_run_rows. The Python layer
 * (various_image_processings_amd/sharded.py) drives the same functions.
 *
 * Geometry (identical on every rank, sharded.py SlabGeometry): rank i owns frame rows
 * [row_begin, row_begin + own) of a frame_height-row frame (balanced contiguous split, the
 * first frame_height % nranks ranks one row more). Its slab is a dense (own + 2r) x width
 * RGB8 buffer (pitch width * 3): rows [0, r) halo above, [r, r + own) own rows,
 * [r + own, 2r + own) halo below, r = ksize / 2 (texture: see below; vip_shard_geometry
 * returns r). The caller fills the own rows; a run
 * receives the halos from the row neighbours, then filters the own rows into `out`
 * (own rows, any pitch). At the first / last rank the missing halo is replaced by the
 * reference's replicate border (reads clamp to the own rows), so the sharded result is
 * bit-identical to one single-GPU launch over the whole frame.
 *
 * Overlap: with vip_shard_set_split(h, 1) a run enqueues the exchange on the shard's own
 * communication stream and, at the same time, the interior rows [r, own - r) (which read
 * only own rows) on the caller's stream; the two r-row edge bands follow once the halos
 * have arrived. The default (split 0) filters all own rows in one launch after the
 * exchange: the two edge launches cost more than a small exchange hides (measured on one
 * MI355X: +11 us per 4K frame at 8 GPUs with two frames in flight, +32 us with one; at
 * radius 15 an edge launch alone exceeds 100 us), and with frames in flight on two
 * streams the exchange of one frame overlaps the other frame's kernel anyway.
 *
 * Transports: RCCL (one communicator per rank; ncclSend/ncclRecv between row neighbours
 * in one group, no collective) or LOCAL (all slabs in one process on one device, halos by
 * device-to-device copies: the same geometry, split and stream ordering, testable on a
 * single GPU).
 *
 * Return value: 0, a hipError_t, a VIP_ERR_* code (vip.h) or VIP_ERR_COMM /
 * VIP_ERR_COMM_TIMEOUT below. Communicator creation never blocks past its timeout: RCCL's
 * initialisation runs on a helper thread, and at the deadline the call returns
 * VIP_ERR_COMM_TIMEOUT, leaving the helper detached (RCCL blocks in its bootstrap while a
 * rank is missing, and aborting such a communicator joins the blocked thread).
 */
#ifndef VIP_SHARD_H
#define VIP_SHARD_H

#include <stddef.h>
#include <stdint.h>

#include "vip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VIP_ERR_COMM 10004         /* an RCCL call failed (vip_shard_last_error) */
#define VIP_ERR_COMM_TIMEOUT 10005 /* communicator set-up not complete before the timeout */
#define VIP_ERR_UNSUPPORTED 10006  /* not available with the RCCL bound in this process */

#define VIP_SHARD_ID_BYTES 128 /* == NCCL_UNIQUE_ID_BYTES */

#define VIP_SHARD_RCCL 0
#define VIP_SHARD_LOCAL 1

typedef struct vip_shard_s* vip_shard_t;

/* Texture filter shards (VIP_FILTER_TEXTURE; vip_shard_create_texture /
 * vip_shard_create_group_texture): the halo is nitr * vip_texture_halo_rows(ksize) rows
 * (45 at k = 5, nitr = 5), exchanged ONCE per frame; iteration t then filters the own
 * rows plus (nitr - 1 - t) * vip_texture_halo_rows(ksize) rows on each side (a ghost zone
 * that shrinks to the own rows), so the result equals one single-GPU vip_texture_run of
 * the whole frame, bit for bit, with one exchange instead of nitr. The shard holds two
 * extra slabs for the iterations, so runs on one texture shard must not overlap (frames in
 * flight on several streams take one shard each, as vip_texture handles do). No
 * interior/edge split (every iteration reads the halo region): vip_shard_set_split(h, 1)
 * returns VIP_ERR_INVALID_ARGUMENT. */

/* Balanced contiguous row split: rank's first row and row count (no device call). */
int vip_shard_rows(int frame_height, int nranks, int rank, int* row_begin, int* own_rows);

/* The communicator id rank 0 creates and the caller broadcasts to every rank
 * (ncclGetUniqueId); `id` holds VIP_SHARD_ID_BYTES bytes. */
int vip_shard_unique_id(void* id);

/* One process per GPU: this rank's shard on the current device, filter kind
 * VIP_FILTER_BILATERAL or VIP_FILTER_ADAPTIVE (vip.h) with the reference's parameters.
 * Every rank calls it with the same id, nranks and filter arguments; it returns once all
 * ranks have joined, or VIP_ERR_COMM_TIMEOUT after timeout_ms (<= 0: 180 s).
 * VIP_ERR_INVALID_ARGUMENT if the thinnest shard is thinner than the halo. */
int vip_shard_create(vip_shard_t* out, int kind, int width, int frame_height, int ksize, float sigma_space,
                     float sigma_color, int numerics, int nranks, int rank, const void* id, int timeout_ms);

/* vip_shard_create for the bilateral texture filter (CudaBilateralTextureFilter's ksize
 * 1..24 and nitr >= 0). */
int vip_shard_create_texture(vip_shard_t* out, int width, int frame_height, int ksize, int nitr, int numerics,
                             int nranks, int rank, const void* id, int timeout_ms);

/* One process, n shards: transport VIP_SHARD_RCCL puts shard i on devices[i] (one RCCL
 * communicator per device, initialised together -- ncclCommInitAll's pattern);
 * VIP_SHARD_LOCAL puts all n on the current device (devices ignored). out[n]. */
int vip_shard_create_group(vip_shard_t* out, int n, int transport, const int* devices, int kind, int width,
                           int frame_height, int ksize, float sigma_space, float sigma_color, int numerics,
                           int timeout_ms);

/* vip_shard_create_group for the bilateral texture filter. */
int vip_shard_create_group_texture(vip_shard_t* out, int n, int transport, const int* devices, int width,
                                   int frame_height, int ksize, int nitr, int numerics, int timeout_ms);

/* 0 (default): one launch over the own rows after the exchange; 1: interior rows during
 * the exchange, then the two edge bands. Same bytes either way. For groups, set it on
 * every member. */
int vip_shard_set_split(vip_shard_t h, int split);

/* Geometry of a shard: its first frame row, own rows and halo rows (r). */
int vip_shard_geometry(vip_shard_t h, int* row_begin, int* own_rows, int* halo_rows);

/* One filter application on this rank's slab (multi-process, RCCL). Asynchronous on
 * `stream`: the slab's own rows must be written before on `stream`; `out` is complete
 * when `stream` is. Every rank must call it once per frame, in the same order. */
int vip_shard_run(vip_shard_t h, uint8_t* d_slab, uint8_t* d_out, size_t out_pitch, void* stream);

/* As vip_shard_run (never from a graph), with timing events (hipEvent_t, timing enabled,
 * as void*): events[0] before the run on `stream`, events[1] after the exchange on the
 * shard's communication stream, events[2] on `stream` after the interior rows (split 1) or
 * once the halos are in (split 0: after `stream`'s wait for them, before the launch),
 * events[3] after the last filter launch on `stream`. */
int vip_shard_run_timed(vip_shard_t h, uint8_t* d_slab, uint8_t* d_out, size_t out_pitch, void* stream,
                        void* const* events);

/* vip_shard_run for n frames at once (slabs[i] -> outs[i]): the halos of all n frames move
 * in ONE RCCL group (its host and device cost is mostly per group: 4 ops ~30 us, 12 ops
 * ~36 us on one MI355X, microbench/rccl_enqueue.hip), then the n filter launches follow
 * on `stream`. Every rank must batch the same frames in the same order. */
int vip_shard_run_batch(vip_shard_t h, int n, uint8_t* const* d_slabs, uint8_t* const* d_outs, size_t out_pitch,
                        void* stream);

/* 0 (default): vip_shard_run_batch launches the filter once per frame; 1: the frames of a
 * batch (split 0, plain or adaptive filter) share launches, up to 6 per launch
 * (vip_bilateral_run_rows_batch / vip_adaptive_run_rows_batch), which leave free_cus CUs to
 * the exchange kernels and the other streams' frames. Same bytes either way; which is
 * faster depends on how the launches meet the exchange kernels (measured per run by
 * bench.py's trial). No effect on the texture filter. */
int vip_shard_set_frames_launch(vip_shard_t h, int on, int free_cus);

/* Graph mode (0 default, 1 on): vip_shard_run captures a frame's whole sequence -- own
 * rows written, the RCCL group on the communication stream, the filter launches -- once per
 * (d_slab, d_out, out_pitch, stream) into a hipGraph and replays it with one hipGraphLaunch
 * (host cost a few us instead of an RCCL group's 16-30 us). The first run of a shard is
 * always direct (RCCL connects its peers lazily, which a capture cannot do), as is any run
 * on the null stream. A shard's communicator must serve one stream at a time: frames in
 * flight on several streams take one shard each. Up to 64 graphs are kept per shard; a
 * change of split or vip_shard_set_graph(h, 0) drops them (waiting on an event the shard
 * owns, so the caller's streams need not outlive the shard). Turning it on returns
 * VIP_ERR_UNSUPPORTED when the RCCL bound in the process is older than 2.27.7 (2.26.6, the
 * copy torch bundles, crashes capturing a send/recv group). If a capture fails, the frame
 * runs directly (its exchange still happens, so the peers are not left waiting), the
 * error goes to stderr and graph mode turns itself off for the shard. */
int vip_shard_set_graph(vip_shard_t h, int on);

/* Number of graphs a shard holds (graph mode). */
int vip_shard_graph_count(vip_shard_t h, int* count);

/* ncclGetVersion of the RCCL bound in this process (e.g. 22707 for 2.27.7). */
int vip_shard_rccl_version(int* version);

/* What the shard's RCCL communicator reports about itself (ncclCommCount,
 * ncclCommUserRank, ncclCommCuDevice): ranks in the communicator, this shard's rank in it,
 * its HIP device. A loopback shard reports 1 / 0 / the current device; a LOCAL shard has no
 * communicator (VIP_ERR_INVALID_ARGUMENT). */
int vip_shard_comm_info(vip_shard_t h, int* count, int* user_rank, int* device);

/* PCI bus id ("dddd:bb:dd.f") of the shard's device (hipDeviceGetPCIBusId); len >= 13. */
int vip_shard_pci_bus_id(vip_shard_t h, char* bus_id, int len);

/* Test transport, one GPU: shard `rank` of an nranks-way geometry whose row neighbours are
 * the shard ITSELF over a one-rank RCCL communicator. The halo above receives the shard's
 * own top halo_rows rows and the halo below its own bottom rows, through the same
 * ncclSend/ncclRecv group, events, split, batch and graph code as a multi-process run, so
 * the result equals the filter of the slab taken as a frame of its own, on its own rows.
 * kind VIP_FILTER_BILATERAL / _ADAPTIVE (sigmas) or VIP_FILTER_TEXTURE (nitr). */
int vip_shard_create_loopback(vip_shard_t* out, int kind, int width, int frame_height, int ksize, float sigma_space,
                              float sigma_color, int nitr, int numerics, int nranks, int rank, int timeout_ms);

/* One filter application of every shard of a group created by vip_shard_create_group
 * (one process): slabs[i], outs[i] (pitch out_pitch) and streams[i] on shard i's device. */
int vip_shard_run_group(vip_shard_t* hs, int n, uint8_t* const* slabs, uint8_t* const* outs, size_t out_pitch,
                        void* const* streams);

/* Text of the last RCCL failure on this thread ("" if none). */
const char* vip_shard_last_error(void);

/* Releases the shard (and its communicator). Group members are destroyed one by one. */
int vip_shard_destroy(vip_shard_t h);

#ifdef __cplusplus
}
#endif

#endif /* VIP_SHARD_H */
