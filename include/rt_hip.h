/* rt_hip.h — C ABI of the gfx950 render path (librtc_amd.so).
 *
 * Boundary it replaces: the body of `void Camera_render(const Camera*, const World*, uint8_t*)`
 * (reference include/raytracing.h:41, src/raytracing.c:86-135).  The reference's only FFI-style
 * seam is that function; the library keeps its symbol (include/raytracing.h) and implements it as
 *     rt_flatten(camera, world)  ->  rt_render(flat, n_gpus, buffer)
 * The lower-level entry points below let a host in any language (ctypes, cgo, JNI: INTEGRATION.md)
 * drive the same kernel with device-resident buffers and its own streams.
 *
 * Conventions: plain C types only, int status (0 = ok, <0 = error, message via rt_last_error()),
 * no torch or HIP types in signatures (streams are passed as void* hipStream_t).
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include "rt_flat.h"
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 1

typedef struct Camera Camera;
typedef struct World World;
typedef struct rt_device_scene rt_device_scene; /* opaque: scene arrays resident in one GPU's HBM */

/* ---- host side: World graph -> flat arrays (replaces the pointer walk of src/raytracing.c:39-84) */
rt_flat_scene *rt_flatten(const Camera *camera, const World *world);
void rt_flat_free(rt_flat_scene *scene);

/* ---- scene presets: the reference driver's scenes 0..7 (src/main.c:9-273, numbering of
 * src/main.c:294-329), built by this library with the reference's defaults (src/main.c:278-287);
 * width <= 0 / spp <= 0 / max_depth <= 0 keep the default (500 / 100 / 50). */
rt_flat_scene *rt_scene_preset(int scene_id, int width, int spp, int max_depth);
/* The same, with relative image file names (scenes 3 and 7: "earthmap.jpg") looked up in image_dir
 * instead of the working directory (NULL: the working directory).  An image that cannot be read
 * (neither a baseline JPEG nor a binary PPM) makes both return NULL with rt_last_error() set; the
 * reference's own Image_new aborts instead (src/texture.c:41), and so does this library's. */
rt_flat_scene *rt_scene_preset_in(int scene_id, int width, int spp, int max_depth, const char *image_dir);

/* ---- device side -------------------------------------------------------------------------- */
int rt_device_count(void);
/* Copy `scene` into HBM of `device` (synchronous, once per render). */
rt_device_scene *rt_scene_upload(const rt_flat_scene *scene, int device);
void rt_scene_release(rt_device_scene *dscene);

/* Render rows row0, row0 + row_stride, ... (n_rows of them) into d_out (device pointer,
 * n_rows * width * 3 bytes, compact, in that row order).  Asynchronous on `stream`
 * (hipStream_t, NULL = default stream of the scene's device): no host synchronisation.  This is
 * the hot path.  Book-1 scenes at >= 64 spp first run a low-spp cost pass (RT_LPT_SPP, default 16)
 * that plans the launch (longest-first order; split pixel streams, rt_book1.h: ChainPx); the image
 * does not depend on the plan.  Launches on one scene share its scratch, so each launch first waits
 * (on the device, hipStreamWaitEvent) for the scene's previous launch, on whatever stream that was;
 * launches on different scenes are independent. */
int rt_render_rows_async(rt_device_scene *dscene, int row0, int row_stride, int n_rows, uint8_t *d_out,
                         void *stream);

/* Completion status of the launches made on dscene since the last call: waits for the scene's last
 * launch, then returns 0 when every work item of its chain launches finished, or -1 (rt_last_error
 * names the number of unfinished items; the frame written is then not valid).  Clears the status.
 * rt_render_rows_async cannot report this itself (it returns before the work runs). */
int rt_scene_check(rt_device_scene *dscene);

/* Whole frame into a host buffer (width*height*3), rows interleaved j mod n_gpus over GPUs
 * 0..n_gpus-1 (n_gpus <= 0: all visible), no collectives.  The host-side preprocessing of the scene
 * runs once; then one host thread per GPU uploads, launches on its own stream, copies its rows back
 * and checks its completion status (rt_scene_check).  Synchronous; 0 only when every pixel of every
 * share was rendered.  This is what Camera_render calls.  RT_REHEARSE_DEVICES=N: run as if N
 * devices were visible (share g on device g % visible count). */
int rt_render(const rt_flat_scene *scene, int n_gpus, uint8_t *out_host);

/* One share of rt_render's partition, for a driver that runs one process (or thread) per GPU (bench.py
 * under torchrun, the cgo / JNI drivers of INTEGRATION.md): rows j % n_shares == share on `device`,
 * written into those rows of out_host (a whole frame's buffer, width*height*3; other rows untouched).
 * Synchronous; 0 only when every pixel of the share was rendered.  Replaces the per-GPU slice of the
 * reference's one `Camera_render` loop (src/raytracing.c:91-135), whose rows the reference's OpenMP
 * team shares out within one process. */
int rt_render_share(const rt_flat_scene *scene, int share, int n_shares, int device, uint8_t *out_host);

/* rt_render and rt_render_share keep each share's device scene (arrays, plan scratch, the record arena),
 * output rows and stream after the call, keyed by the scene's bytes, the partition and the RT_*
 * environment: a repeated call with the same scene renders without upload or allocation (DESIGN.md
 * §5.3).  One partition per device is kept; RT_SCENE_CACHE=0 keeps nothing.  This frees what is kept
 * (call it before freeing device memory for other work; in-flight calls finish first). */
void rt_render_cache_release(void);

/* Kernel-side timing of the last rt_render call on `device`: milliseconds between HIP events
 * bracketing its kernel launches (excludes upload and D2H). */
double rt_last_kernel_ms(int device);

/* Host wall-clock phases of the last rt_render / rt_render_share of share `share` (ms[4]): setup
 * (upload and allocations; ~0 when the cached scene was reused), launch to finish (pre-pass, plan,
 * kernels), D2H of its rows with the completion check, and the whole call. */
int rt_last_share_ms(int share, double *ms);

/* Diagnostics: evaluate the device libm port (rt_libm.h) on n inputs.
 * fn: 0 = sincosf (out[2i] = sin, out[2i+1] = cos), 1 = powf(x, 5), 2 = logf, 3 = sinf,
 *     4 = atan2f(x[2i], x[2i+1]) into out[i] (n = 2 * pairs), 5 = acosf. */
int rt_diag_libm(int fn, const float *x_host, float *out_host, int64_t n, int device);

/* Diagnostics: bitwise checks of the Book-1 kernel's exact arithmetic cores against the compiler's
 * sqrtf / division on the device (fn 0: sqrt over float bit patterns start..start+count-1,
 * fn 1: division on `count` hashed pairs, fn 2: the sphere-hit outcome on hashed rays);
 * *mismatches receives the number of differing results. */
int rt_diag_arith(int fn, uint64_t start, uint64_t count, uint64_t seed, unsigned long long *mismatches, int device);

/* Milliseconds of the last frame launch rt_render_rows_async made for `dscene` (HIP events on its
 * stream; call after that work completed).  Excludes the cost pre-pass and the plan
 * (rt_book1_cost_kernel, chain_* planner kernels).  -1 when unavailable.  Since r05 the pre-pass renders
 * each pixel's first samples (up to 64) and the frame launch goes on from them, so this excludes part of
 * the frame's sample work: compare whole steps (pre-pass + plan + frame launch + fold) across builds,
 * not this number (bench.py's roofline uses the step time). */
double rt_scene_last_launch_ms(rt_device_scene *dscene);

/* The same for the scene's last min(max, 64) launches, oldest first, into ms[]: returns how many were
 * written (-1 on error; a launch whose kernels record no bracket, e.g. a deep-path launch, reads -1).
 * bench.py reports their spread (min / p50 / max per step). */
int rt_scene_launch_history(rt_device_scene *dscene, double *ms, int max);

/* Diagnostics (RT_PX_TIME=1 set at upload time): the last chain launch, one row of 16 uint32 per work
 * item in item order: pixel, segment, K, whole-wave (1) / lane (0), start, end (wall_clock64 ticks,
 * 100 MHz, low 32 bits), records written (samples for segment 0 / unsplit), flags (bit 0 coupled,
 * bit 1 ended), link segment, link record, segment length (draws), the pixel's pre-pass draws, the
 * pixel's own pre-pass cost (traversal steps), the tick at which a helper wave took the item over (tail
 * migration; 0: never migrated), the planner's cost of the pixel (max(own, row-neighbour mean) when
 * cost smoothing is on, else the own cost), where the item started (XCC_ID << 28 | HW_ID bits 0-15: wave,
 * SIMD, pipe, CU, SH, SE; 0 for items a helper started).
 * Returns the number of items (at most max_rows rows are written), -1 on error. */
int64_t rt_scene_chain_diag(rt_device_scene *dscene, uint32_t *rows, int64_t max_rows);

/* Name of the frame kernel rt_render_rows_async launches for `dscene` over its whole image (as
 * rocprofv3 lists it). */
const char *rt_scene_kernel(const rt_device_scene *dscene);

const char *rt_last_error(void);
int rt_abi_version(void);
/* A hash of the library's sources and compile flags (16 hex digits): profiles under profiles/ record
 * the id of the build they measured, and bench.py attaches their counters only to that build. */
const char *rt_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* RT_HIP_H */
