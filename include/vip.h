/*
 * vip.h — C ABI of the MI355X-native bilateral-filter family.
 *
 * Drop-in boundary for the reference's include/cuda/ headers' API
 * (yuyuyu-bot/various_image_processings). Plain pointers and sizes only; every
 * image pointer is a DEVICE pointer to dense interleaved 8-bit 3-channel data
 * (or f32 where stated). `pitch` arguments are row strides in bytes; the
 * reference API has no pitch, so its wrappers pass width*channels*sizeof(T).
 * `stream` is a hipStream_t (NULL = the legacy default stream). Every run
 * function is asynchronous on `stream`: the C++ wrappers in include/cuda/ add
 * the device synchronisation the reference performs in its public methods.
 *
 * Return value: 0 on success, otherwise a hipError_t code, or one of the
 * VIP_ERR_* codes below for argument errors (the reference printed launch errors
 * to stderr and carried on, src/host_utilities.hpp:9-13).
 */
#ifndef VIP_H
#define VIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VIP_ABI_VERSION 1

/* numerics profile */
#define VIP_NUMERICS_CUDA 0 /* as src/<filter>_impl.cu: float-coefficient LUTs, fused multiply-add accumulate */
#define VIP_NUMERICS_CPP 1  /* as include/cpp/<filter>.hpp: double-coefficient LUTs, separate multiply and add */

/* argument errors (hipError_t values stay below 1000) */
#define VIP_ERR_INVALID_ARGUMENT 10001 /* null handle/pointer, non-positive size */
#define VIP_ERR_UNSUPPORTED_KSIZE 10002 /* ksize outside what the reference runs: see vip_max_ksize */
#define VIP_ERR_ALIASING 10003 /* dst aliases src or guide (the kernels read neighbours other blocks write) */

typedef struct vip_bilateral_s* vip_bilateral_t;
typedef struct vip_adaptive_s* vip_adaptive_t;
typedef struct vip_texture_s* vip_texture_t;

int vip_abi_version(void);
/* The kernels the calling thread launched through this library since its previous call,
 * as the profiler names them ("void vip::bilateral_kernel<7, 16, ...>", no parameter
 * list), newline-separated, each once. With a buffer (len > 0) it writes at most len - 1
 * bytes and a terminating 0 and clears the list; buf = NULL, len = 0 only returns the
 * length. Returns the full length. No reference counterpart: it lets a benchmark
 * name the exact template instantiation it timed. */
int vip_launched_kernels(char* buf, size_t len);
/* Kernel-duration recorder of the calling thread (measurement; no reference counterpart).
 * After vip_kernel_timing_begin(capacity) the next `capacity` kernels this thread launches
 * through the library carry a (start, stop) event pair that the runtime stamps with the
 * kernel's own begin and end (hipExtLaunchKernel): no marker packet enters the stream, so a
 * duration is what rocprofv3 --kernel-trace reports for that launch. Begin clears earlier
 * records (capacity 1..65536). vip_kernel_timing_end() stops recording and returns the
 * number of launches recorded. vip_kernel_timing_get(i, &ms, name, len), after end, waits
 * for launch i to finish and returns its duration and (if name) its kernel name as
 * vip_launched_kernels names it. */
int vip_kernel_timing_begin(int capacity);
int vip_kernel_timing_end(void);
int vip_kernel_timing_get(int index, float* ms, char* name, size_t len);
const char* vip_error_string(int code);
/* Largest filter radius (ksize/2) any filter accepts (32: bilateral ksize 65). */
int vip_max_radius(void);

/* Largest ksize each filter accepts: what the reference runs. Its kernels size dynamic
 * shared memory from ksize with no cap against CUDA's 48 KB default
 * (src/bilateral_filter_impl.cu:252-254, 272-275; src/adaptive_bilateral_filter_impl.cu:165-167),
 * so: bilateral 65, joint bilateral 47, adaptive 63, texture 24 (its JBF is 2k-1 <= 47).
 * Bilateral, joint and adaptive take odd ksize from 1 (radius 0: output = input for
 * sigma_space > 0); the texture filter any ksize from 1. The C++ and Python layers take
 * the same sets. Returns VIP_ERR_INVALID_ARGUMENT for an unknown filter. */
#define VIP_FILTER_BILATERAL 0
#define VIP_FILTER_JOINT 1
#define VIP_FILTER_ADAPTIVE 2
#define VIP_FILTER_TEXTURE 3
int vip_max_ksize(int filter);

/* Kernel selection, process-wide (no reference counterpart; results are identical either
 * way). AUTO: radius-specialised kernels for radius 1..15, the runtime-radius kernel for
 * radius 0 and 16..32. RUNTIME: the runtime-radius kernel for every radius (test and
 * measurement knob). The environment variable VIP_STENCIL_PATH=1 sets RUNTIME at load. */
#define VIP_PATH_AUTO 0
#define VIP_PATH_RUNTIME 1
int vip_set_stencil_path(int path);

/* ---- device buffers: replaces DeviceImage<T> (include/cuda/device_image.hpp:4-16,
 *      src/device_image.cu:5-52) ---- */
int vip_malloc(void** d_ptr, size_t bytes);
int vip_free(void* d_ptr);
int vip_upload(void* d_dst, const void* h_src, size_t bytes);   /* blocking H2D */
int vip_download(void* h_dst, const void* d_src, size_t bytes); /* blocking D2H */
int vip_device_synchronize(void);
int vip_stream_synchronize(void* stream);
/* Device selection for multi-GPU callers (the reference drives the implicit current
 * device only): every handle, buffer and launch belongs to the calling thread's
 * current device at the time of the call. */
int vip_device_count(int* count);
int vip_set_device(int device);
int vip_get_device(int* device);

/* ---- host-frame path (the reference's DeviceImage::upload/download,
 *      src/device_image.cu:10-16, copy pageable memory synchronously through thrust).
 *      Pinned host frames + stream-ordered copies let H2D, kernels and D2H of
 *      successive frames overlap on separate streams. ---- */
int vip_host_alloc(void** h_ptr, size_t bytes);  /* page-locked host memory */
int vip_host_free(void* h_ptr);
int vip_upload_async(void* d_dst, const void* h_src, size_t bytes, void* stream);   /* stream-ordered H2D */
int vip_download_async(void* h_dst, const void* d_src, size_t bytes, void* stream); /* stream-ordered D2H */
int vip_stream_create(void** stream);  /* non-blocking HIP stream, returned as void* */
int vip_stream_destroy(void* stream);
/* Cross-stream ordering for a split pipeline (one upload, one compute and one download
 * stream): H2D and D2H on their own streams overlap (measured 0.52 ms per 4K frame
 * pair vs 0.89 ms when one stream carries both directions). No timing. */
int vip_event_create(void** event);
int vip_event_destroy(void* event);
int vip_event_record(void* event, void* stream);
int vip_stream_wait_event(void* stream, void* event); /* later work on stream waits for event */
int vip_event_synchronize(void* event);               /* host waits for event */

/* ---- bilateral / joint bilateral: CudaBilateralFilter
 *      (include/cuda/bilateral_filter.hpp:9-24, src/bilateral_filter_impl.cu:204-310) ---- */
int vip_bilateral_create(vip_bilateral_t* out, int width, int height, int ksize, float sigma_space,
                         float sigma_color, int numerics);
int vip_bilateral_destroy(vip_bilateral_t h);
/* Impl::bilateral_filter (:241-258) */
int vip_bilateral_run(vip_bilateral_t h, const uint8_t* d_src, size_t src_pitch, uint8_t* d_dst, size_t dst_pitch,
                      void* stream);
/* Impl::joint_bilateral_filter (:260-280): colour weights from d_guide, sums of d_src */
int vip_joint_bilateral_run(vip_bilateral_t h, const uint8_t* d_src, size_t src_pitch, const uint8_t* d_guide,
                            size_t guide_pitch, uint8_t* d_dst, size_t dst_pitch, void* stream);
/* Row-band variant for row-sharded frames (no reference counterpart; multi-GPU C5).
 * Filters `out_rows` rows of a handle-width image. Output row i is centred on source
 * row i + src_row0; neighbour rows are clamped to [row_lo, row_hi) of d_src, with
 * 0 <= row_lo < row_hi <= the handle's height (d_src and d_guide hold that many rows;
 * rows below row_lo / above row_hi-1 replicate them, which is exactly the reference's
 * replicate border at the frame edges). d_guide may be NULL (plain bilateral).
 * Returns VIP_ERR_INVALID_ARGUMENT for a row range outside the handle's rows. */
int vip_bilateral_run_rows(vip_bilateral_t h, const uint8_t* d_src, size_t src_pitch, const uint8_t* d_guide,
                           size_t guide_pitch, uint8_t* d_dst, size_t dst_pitch, int out_rows, int src_row0,
                           int row_lo, int row_hi, void* stream);
/* n frames of the same geometry (no reference counterpart; a shard's frames per RCCL group,
 * vip_shard_run_batch): frame f filters d_srcs[f] into d_dsts[f] exactly as
 * vip_bilateral_run_rows(h, d_srcs[f], src_pitch, NULL, 0, d_dsts[f], dst_pitch, out_rows,
 * src_row0, row_lo, row_hi, stream) would, with up to 6 frames per launch: the persistent
 * workgroups run from one frame's tiles into the next one's, so a small slab's launch
 * prologue and tail are paid once per launch. free_cus >= 0: CUs the launch leaves to
 * concurrent work (another stream's frames, an exchange kernel); 0 = all CUs.
 * VIP_ERR_ALIASING when any d_dsts[f] equals any d_srcs[g]. Results are identical to the
 * per-frame calls. */
int vip_bilateral_run_rows_batch(vip_bilateral_t h, int n, const uint8_t* const* d_srcs, size_t src_pitch,
                                 uint8_t* const* d_dsts, size_t dst_pitch, int out_rows, int src_row0, int row_lo,
                                 int row_hi, int free_cus, void* stream);
/* Tuning knob, process-wide (no reference counterpart): waves per workgroup of the plain
 * bilateral kernel for radius <= 8. 0 (default) = chosen per launch from the frame's
 * tile count (small frames take 8 or 4 waves and smaller tiles so more CUs work);
 * 16, 8 or 4 forces one. Results are identical for every setting (only the tiling
 * changes). The environment variable VIP_BIL_WAVES sets the initial value. */
int vip_bilateral_set_waves(int waves);
/* Companion knob: the tile shape of the same kernel for radius <= 8. 0 (default) = chosen
 * per launch with the wave count (small frames and the slabs of a frame split over many
 * GPUs take 256-pixel tiles, one row per wave and 4 outputs per thread: half the serial
 * work per thread); 1 forces 128-pixel tiles (4 rows per wave, 8 outputs per thread),
 * 2 forces 256-pixel tiles. Results are identical for every setting. The environment
 * variable VIP_BIL_WIDE sets the initial value. A forced wave count with mode 0 keeps
 * 128-pixel tiles. */
int vip_bilateral_set_wide(int mode);
/* Frames in flight the same choice plans for: 0 (default) = counted per device from the
 * distinct streams among its last 8 plain-bilateral launches (at most 4), so frames in
 * flight on several streams each get a tiling sized for their share of the CUs; 1..4 forces
 * the count (a measurement knob: e.g. timing one frame alone with the tiling the in-flight
 * frames use). The count is of streams, not of launches outstanding: a caller that
 * alternates streams but waits for each frame counts 2 or more too, and should force 1.
 * Results are identical for every setting. */
int vip_bilateral_set_frames_in_flight(int n);

/* ---- adaptive bilateral: CudaAdaptiveBilateralFilter
 *      (include/cuda/adaptive_bilateral_filter.hpp:9-19, src/adaptive_bilateral_filter_impl.cu:117-191) ---- */
int vip_adaptive_create(vip_adaptive_t* out, int width, int height, int ksize, float sigma_space, float sigma_color,
                        int numerics);
int vip_adaptive_destroy(vip_adaptive_t h);
int vip_adaptive_run(vip_adaptive_t h, const uint8_t* d_src, size_t src_pitch, uint8_t* d_dst, size_t dst_pitch,
                     void* stream);
int vip_adaptive_run_rows(vip_adaptive_t h, const uint8_t* d_src, size_t src_pitch, uint8_t* d_dst, size_t dst_pitch,
                          int out_rows, int src_row0, int row_lo, int row_hi, void* stream);
/* n frames per launch (up to 6), as vip_bilateral_run_rows_batch */
int vip_adaptive_run_rows_batch(vip_adaptive_t h, int n, const uint8_t* const* d_srcs, size_t src_pitch,
                                uint8_t* const* d_dsts, size_t dst_pitch, int out_rows, int src_row0, int row_lo,
                                int row_hi, int free_cus, void* stream);

/* ---- gradient magnitude: cuda_gradient<T> (include/cuda/gradient.hpp:4-23, src/gradient_impl.cu:90-112) ---- */
int vip_gradient_u8(const uint8_t* d_src, float* d_dst, int width, int height, int src_ch, int numerics,
                    void* stream);
int vip_gradient_f32(const float* d_src, float* d_dst, int width, int height, int src_ch, int numerics,
                     void* stream);

/* ---- bilateral texture filter: CudaBilateralTextureFilter
 *      (include/cuda/bilateral_texture_filter.hpp:7-17, src/bilateral_texture_filter_impl.cu:179-275) ---- */
int vip_texture_create(vip_texture_t* out, int width, int height, int ksize, int nitr, int numerics);
int vip_texture_destroy(vip_texture_t h);
/* Device bytes a texture handle of this frame size allocates for its frames: two
 * ping-pong frames and the guide, u8x3 each (the reference's Impl also held f32
 * magnitude, blurred and rtv buffers, 20 B/px; no f32 scratch is held here). */
size_t vip_texture_scratch_bytes(int width, int height);
/* Impl::execute (:199-214); d_src and d_dst are dense width*3. The handle owns scratch
 * frames (like the reference's Impl): runs on one handle must not overlap, so frames in
 * flight on several streams take one handle per stream. Bilateral and adaptive handles
 * hold only read-only LUTs and may run on several streams at once. */
int vip_texture_run(vip_texture_t h, const uint8_t* d_src, uint8_t* d_dst, void* stream);
/* vip_texture_run with per-stage timestamps (measurement; no reference counterpart):
 * `events` holds 2*nitr + 1 hipEvent_t (created with timing enabled, passed as void*);
 * events[2i] is recorded on `stream` before iteration i's guide stage, events[2i+1]
 * before its joint bilateral, events[2*nitr] after the last launch. */
int vip_texture_run_timed(vip_texture_t h, const uint8_t* d_src, uint8_t* d_dst, void* stream, void* const* events);

/* Iteration form (no reference counterpart; same bytes either way). TWO_LAUNCH (the
 * default): per iteration the fused guide stage writes the guide frame to HBM and the
 * joint bilateral reads it -- src/bilateral_texture_filter_impl.cu:207-210's four stages
 * in two launches. FUSED (ksize 5 only, else VIP_ERR_UNSUPPORTED_KSIZE): one launch per
 * iteration, the guide of each JBF tile computed in LDS with the JBF apron (SURVEY
 * §8(f)1); vip_texture_run_timed's events[2i+1] then follows the whole iteration. The
 * row-slab entry point below always uses TWO_LAUNCH. */
#define VIP_TEXTURE_TWO_LAUNCH 0
#define VIP_TEXTURE_FUSED 1
int vip_texture_set_mode(vip_texture_t h, int mode);

/* Row-slab form of one texture iteration for a row-sharded frame (SURVEY §8(f)3;
 * the reference is single-GPU). d_src is a dense slab of the handle's width x
 * height (pitch width*3) whose rows [row_lo, row_hi) are valid frame rows: every
 * stage clamps into them, which at a frame edge is the reference's replicate
 * border. Writes the iteration's rows [out_row0, out_row0 + out_rows) to d_dst
 * (row 0 of d_dst = slab row out_row0). Rows further than vip_texture_halo_rows(k)
 * from the frame edge must be backed by valid neighbour rows in d_src. */
int vip_texture_halo_rows(int ksize);
int vip_texture_iterate_rows(vip_texture_t h, const uint8_t* d_src, uint8_t* d_dst, size_t dst_pitch, int out_row0,
                             int out_rows, int row_lo, int row_hi, void* stream);
/* Impl::compute_blur_and_rtv (:216-237): image u8x3, magnitude f32 -> blurred f32x3, rtv f32 */
int vip_texture_blur_rtv(vip_texture_t h, const uint8_t* d_image, const float* d_magnitude, float* d_blurred,
                         float* d_rtv, void* stream);
/* Impl::compute_guide (:239-256): blurred f32x3, rtv f32 -> guide u8x3 */
int vip_texture_guide(vip_texture_t h, const float* d_blurred, const float* d_rtv, uint8_t* d_guide, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* VIP_H */
