/*
 * rt_api.h -- C ABI of the MI355X-native render path for erichgess/rust_tracer.
 *
 * This is the drop-in boundary.  It replaces the reference's Rust seam
 *
 *     pub fn render(camera: &Camera, scene: &Scene, buffer: &mut RenderBuffer, depth: usize)
 *                                                                    (src/render.rs:31-38)
 *
 * with a flat, insertion-ordered scene description (what src/scene/mod.rs:40-52
 * `add_shape` / `add_light` / `set_ambient` accumulate), a camera record
 * (src/render.rs:155-176) and caller-owned output buffers.  Everything is plain C:
 * pointers, sizes, int32 status codes.  No torch or HIP types appear in the
 * signatures; streams are passed as opaque `void*` (a hipStream_t).
 *
 * Conventions
 *  - All entry points return rt_status (0 = RT_OK).  The reference panics instead
 *    (Matrix::invert "Singular Matrix", src/math/matrix.rs:116-117); here the panic
 *    becomes RT_ERR_SINGULAR_MATRIX from rt_scene_create.
 *  - The library owns device memory; the caller owns host buffers.
 *  - An rt_scene handle is not safe for concurrent rt_render calls (mirrors the
 *    reference's !Sync Rc<RefCell<..>> scene).
 *  - Output is row-major [v][u][rgb] float32 (image order).  The reference buffer is
 *    column-major `buf[u][v]` (src/render.rs:5-19); INTEGRATION.md shows the
 *    transposing copy a Rust binding does.
 */
#ifndef RT_API_H
#define RT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_API_VERSION 1

typedef int32_t rt_status;
enum {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = 1,
    RT_ERR_SINGULAR_MATRIX = 2,  /* src/math/matrix.rs:116-117 panic("Singular Matrix") */
    RT_ERR_UNSUPPORTED = 3,      /* e.g. depth above RT_MAX_DEPTH */
    RT_ERR_NO_DEVICE = 4,        /* no HIP device / HIP runtime failure at init */
    RT_ERR_HIP = 5,              /* a HIP runtime call failed */
    RT_ERR_OUT_OF_MEMORY = 6,
    RT_ERR_BAD_MATERIAL = 7,     /* material index out of range */
    RT_ERR_CAPACITY = 8          /* a ray queue overflowed its pool: the frame is incomplete
                                    (render.rs:40-103 traces every ray; this build never
                                    returns a truncated frame as RT_OK) */
};

/* Largest `depth` the device path accepts (the reference recursion is unbounded; its
 * ray trees end where every branch missed, which the level-synchronous pipeline detects:
 * rt_render stops enqueuing levels once one is empty). */
#define RT_MAX_DEPTH 1024
#define RT_MAX_LIGHTS 65536 /* lights per scene (the shadow-queue keys hold a 16-bit light index; above
                               256 lights a shadow entry takes 8 B: node and light side by side).
                               Each node keeps one bit per light: ceil(lights / 32) words */

/* ---------------------------------------------------------------- scene description */

typedef struct rt_color {
    float r, g, b;                 /* src/scene/color.rs:2-6 */
} rt_color;

/* Texture programs.  The reference stores host fn pointers (`ColorFun`,
 * src/scene/material.rs:3) -- a GPU needs a closed set.  Every texture used by the
 * reference's scenes is one of these:
 *   RT_TEX_CONST         -> `color`                          (Phong fields; dim_white
 *                                                             = 0.1*WHITE, my_scene.rs:11-13)
 *   RT_TEX_CHECKERBOARD  -> my_scene.rs:26-43 (WHITE / 0.5*WHITE), `color` unused      */
enum { RT_TEX_CONST = 0, RT_TEX_CHECKERBOARD = 1 };
typedef struct rt_texture {
    int32_t kind;
    rt_color color;
} rt_texture;

/* Materials (src/scene/material.rs).  PHONG uses the three CONST colours
 * (`Phong::new(ambient, diffuse, specular, power, reflectivity, refraction_index)`,
 * material.rs:35-51); TEXTURE_PHONG evaluates the texture programs at the hit's
 * texture coordinates (material.rs:113-130, 144-186). */
enum { RT_MAT_PHONG = 0, RT_MAT_TEXTURE_PHONG = 1 };
typedef struct rt_material {
    int32_t kind;
    rt_texture ambient;
    rt_texture diffuse;
    rt_texture specular;
    float power;
    float reflectivity;
    float refraction_index;
} rt_material;

/* Shapes, in Scene::add_shape order (that order is the nearest-hit tie-break,
 * src/scene/mod.rs:98-116).
 *   SPHERE   : unit sphere at the origin + `transform` (sphere.rs:57-103)
 *   PLANE    : data[0..3] origin, data[3..6] normal (plane.rs:22-42) + `transform`
 *   TRIANGLE : data[0..9] = v0, v1, v2 (triangle.rs:16-39); `transform` is stored
 *              but, as in the reference, ignored by intersect (triangle.rs:51-99)
 *   CUBE     : unit cube of 12 triangles (cube.rs:21-77) + `transform`
 * `transform` is the row-major forward matrix handed to `set_transform`
 * (matrix.rs:16-20; identity when never set).  The library inverts it with the
 * reference's Gauss-Jordan (matrix.rs:99-153). */
enum { RT_SHAPE_SPHERE = 0, RT_SHAPE_PLANE = 1, RT_SHAPE_TRIANGLE = 2, RT_SHAPE_CUBE = 3 };
typedef struct rt_shape {
    int32_t kind;
    int32_t material;              /* index into rt_scene_desc.materials */
    float transform[16];           /* row-major 4x4 */
    float data[9];
} rt_shape;

/* Lights (src/scene/mod.rs:169-246). */
enum { RT_LIGHT_POINT = 0, RT_LIGHT_AMBIENT = 1 };
typedef struct rt_light {
    int32_t kind;
    float pos[3];                  /* POINT only */
    rt_color color;
} rt_light;

typedef struct rt_scene_desc {
    uint32_t n_materials;
    const rt_material* materials;
    uint32_t n_shapes;
    const rt_shape* shapes;
    uint32_t n_lights;             /* at most RT_MAX_LIGHTS (more -> RT_ERR_UNSUPPORTED from
                                      rt_scene_create*; the reference has no limit,
                                      scene/mod.rs:189-206 loops over all) */
    const rt_light* lights;
    rt_color ambient;              /* Scene::set_ambient (mod.rs:50-52) */
} rt_scene_desc;

/* src/render.rs:155-176.  Camera::new(x_res, y_res) is origin (0,0,-8), window [-3,3]^2. */
typedef struct rt_camera {
    float origin[3];
    float x_min, x_max, y_min, y_max;
    uint32_t x_res, y_res;
} rt_camera;

/* ---------------------------------------------------------------- render options */

typedef struct rt_counters {
    uint64_t node_rays;     /* scene scans for primary/reflected/refracted rays
                               (Scene::intersect from trace_ray, render.rs:47) */
    uint64_t shadow_rays;   /* scene scans for point-light shadow rays (mod.rs:193) */
    uint64_t pixels;        /* pixels rendered by this call */
    uint64_t wave_iterations; /* reserved, 0 (the per-pixel megakernel of round 1 counted its
                                 loop iterations here; the level pipeline does not) */
} rt_counters;

typedef struct rt_render_opts {
    int32_t device;          /* HIP device ordinal; -1 = current device */
    rt_counters* counters;   /* optional out: ray counters of this call */
    float* kernel_ms;        /* optional out: device time of the render kernel (HIP events) */
} rt_render_opts;

/* ---------------------------------------------------------------- entry points */

typedef struct rt_scene rt_scene;

/* Copies and flattens `desc`, runs the host-side preprocessing the reference does at
 * scene build time (Matrix::inverse, Plane axes, Triangle normals, Cube triangles) and
 * uploads the scene to `device` (-1 = current). */
rt_status rt_scene_create(const rt_scene_desc* desc, int32_t device, rt_scene** out);
/* rt_scene_create with explicit tuning: "key=value" pairs separated by ',' (the keys of
 * rust_tracer_amd/csrc/rt_tune.hpp, e.g. "lb_res=0,bvh=0").  Every key is exact -- it moves
 * time, never a pixel.  A handle's tuning is the defaults, then the environment's RT_TUNE
 * (same syntax; the library's only environment read), then `tuning`; clones copy it.  An
 * unknown key or a bad value is RT_ERR_INVALID_ARG.  tuning == NULL is rt_scene_create. */
rt_status rt_scene_create_tuned(const rt_scene_desc* desc, int32_t device, const char* tuning, rt_scene** out);
/* Changes the per-pass keys of rt_tune.hpp on a handle (and its band shares / devices);
 * scene-build keys are RT_ERR_INVALID_ARG here.  Not while a render of the handle runs. */
rt_status rt_scene_set_tuning(rt_scene* scene, const char* tuning);
rt_status rt_scene_destroy(rt_scene* scene);
/* The host half of rt_scene_create alone (no HIP call, no device needed): builds the image
 * the scene's device allocation would hold for `desc` under `tuning` and returns its FNV-1a
 * digest and size in bytes.  A check that the scene build is deterministic (e.g. the same
 * image for any build_threads), and a way to time the build on a machine without a GPU. */
rt_status rt_scene_layout_digest(const rt_scene_desc* desc, const char* tuning, uint64_t* digest,
                                 uint64_t* bytes);

/* Page-locked host memory for a caller's frame buffer (the RenderBuffer a render() caller
 * owns, render.rs:5-19): rt_render's device-to-host copy of the frame then runs at the
 * link's DMA rate instead of through a pageable staging copy.  Any host pointer stays
 * valid for rt_render; this is an optional fast path.  rt_host_free releases it. */
rt_status rt_host_alloc(uint64_t bytes, void** out);
rt_status rt_host_free(void* ptr);

/* A second handle of the same scene on `device` (-1 = current), copied device-to-device (no
 * host rebuild): its own workspace and stream, so two handles can render concurrently
 * (frames in flight) or on two GPUs. */
rt_status rt_scene_clone(const rt_scene* src, int32_t device, rt_scene** out);

/* Multi-GPU render behind the same seam.  One host thread drives
 * every listed device: the scene is built once and uploaded to each device; rt_render /
 * rt_render_spp on the returned handle deal the frame's rows in block-cyclic bands of 8
 * over the devices (band b -> devices[b % n]), render them concurrently, gather the bands
 * on devices[0] with RCCL (ncclGather over xGMI, communicators from ncclCommInitAll) and
 * un-permute them there before the copy to the caller's buffers.  The result equals the
 * one-device rt_render bit for bit (pixels are independent).  n_devices == 1 is
 * rt_scene_create, unless the handle's tuning sets force_rccl=1 (RT_TUNE): then the one device gets a
 * one-rank RCCL communicator and renders go through the same band render, ncclGather and
 * un-permute as n > 1 (a one-GPU machine runs the RCCL exchange this way).  A device listed twice shares that GPU between two band shares, which
 * then exchange bands by device copies (RCCL puts one rank per device; a test
 * configuration).  The stream-ordered entry points act on devices[0] only. */
rt_status rt_scene_create_multi(const rt_scene_desc* desc, const int32_t* devices, uint32_t n_devices,
                                rt_scene** out);

/* Device bytes the scene's render workspace holds now (node pool, ray and shadow queues,
 * sort buffers, frame buffers of rt_render): it grows with the largest pass rendered so far
 * (pixels x frames per pass x RT_NODE_FACTOR node slots) and after a reported overflow. */
uint64_t rt_scene_workspace_bytes(const rt_scene* scene);

/* Devices a scene renders on (1 unless made by rt_scene_create_multi), and whether its band
 * exchange runs over RCCL. */
int32_t rt_scene_device_count(const rt_scene* scene);
int32_t rt_scene_uses_rccl(const rt_scene* scene);

/* render.rs:31-38: fill `rgb` (h*w*3 float, row-major [v][u][c]) with
 * trace_ray(get_ray(u, v), depth) for every pixel.  `rgb8` (optional, may be NULL)
 * receives Color::as_u8 (color.rs:43-46) of every pixel, row-major RGB8.
 * On a one-device scene the frame is rendered as two contiguous row shares side by side on
 * two streams (RT_SEAM_SPLIT, default 2; 1 = one pass), each copied from its own stream
 * straight into `rgb` / `rgb8`; the row where the shares meet follows their finish times
 * from call to call (RT_SEAM_ADAPT; RT_SEAM_BAND_ROWS pins it) and their persistent grids
 * take RT_SEAM_GRID_PCT (default 80) % of the chip.  None of this changes a pixel. */
rt_status rt_render(const rt_scene* scene, const rt_camera* camera, uint32_t depth,
                    const rt_render_opts* opts, float* rgb, uint8_t* rgb8);

/* Device-resident variant used by the multi-GPU driver: renders this rank's share of
 * the frame into device memory on `stream`, asynchronously.
 * Rows are dealt in bands of `band_rows`: band b (rows [b*band_rows, (b+1)*band_rows))
 * belongs to rank b % world.  This rank's bands are written back to back into
 * `d_rgb` (band-major, rows of x_res*3 floats), rt_band_rows_per_rank() rows in all
 * (the last bands are padded; padded rows are written as 0).
 * Stream-ordered: a ray-queue overflow is reported later by rt_scene_sync_status.
 * `d_counters` (optional) is a device array of 3 uint64 that the kernel ADDS
 * node_rays, shadow_rays, pixels into. */
rt_status rt_render_bands_async(const rt_scene* scene, const rt_camera* camera,
                                uint32_t depth, uint32_t band_rows, uint32_t rank,
                                uint32_t world, float* d_rgb, uint64_t* d_counters,
                                void* stream);

/* render.rs:31-38 in stream order: the whole frame, row-major, into device memory (`d_rgb`:
 * y_res*x_res*3 floats; `d_rgb8` optional, Color::as_u8 bytes; `d_counters` optional, 3
 * uint64 the kernels ADD node_rays, shadow_rays, pixels into), enqueued on `stream` without
 * a host round trip.  rt_render's seam split on a one-device scene: two contiguous row
 * shares render side by side on rt_render's two internal streams (the scene and one clone,
 * each with its own workspace), forked from and joined back into `stream`; RT_SEAM_SPLIT=1
 * or y_res < 32: one pass on `stream`.  Bit-identical to rt_render.  A queue overflow is
 * reported by rt_scene_sync_status (the frame is then incomplete; render it again), also
 * when an rt_render on the same scene ran in between.  Pass a created stream: on the legacy
 * null stream the fork and join serialise with the process's other streams (measured 5.4
 * instead of 3.4 ms per 1080p frame).  One-device scenes
 * only (RT_ERR_UNSUPPORTED on rt_scene_create_multi's).  No reference counterpart beyond
 * render() itself: the device-resident form of the seam. */
rt_status rt_render_frame_async(const rt_scene* scene, const rt_camera* camera, uint32_t depth,
                                float* d_rgb, uint8_t* d_rgb8, uint64_t* d_counters, void* stream);

/* Frame batch: n_frames (1..rt_max_frames() = 32) frames of one resolution, each with its own camera, in one
 * pipeline pass (the per-level launch and latency floor is paid once per batch).  The ray
 * queues of a batch are ordered by ray alone -- rays of different frames that start in the
 * same place and head the same way share waves (an ordering property only: each task
 * carries its frame; level 0 is frame-uniform per wave); RT_FRAME_KEYS=frame keeps each
 * frame contiguous instead (the frame index above every key bit).  d_rgb holds n_frames
 * consecutive band buffers of rt_band_rows_per_rank(y_res, band_rows, world) x x_res x 3
 * floats; each equals rt_render_bands_async of that frame's camera bit for bit.  No
 * reference counterpart: a throughput form of render() (src/render.rs:31) over frames. */
rt_status rt_render_bands_batch_async(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames,
                                      uint32_t depth, uint32_t band_rows, uint32_t rank, uint32_t world,
                                      float* d_rgb, uint64_t* d_counters, void* stream);

/* The general stream-ordered render (every *_async render above is a special case of it):
 * n_frames (1..rt_max_frames() = 32) frames of one resolution, each with its own camera, spp jittered samples
 * per pixel (spp > 1 needs n_frames == 1), this rank's row bands (as rt_render_bands_async).
 *  - d_rgb:  n_frames band buffers of f32 RGB (may be NULL when spp == 1 and d_rgb8 is set:
 *            then only the bytes are written);
 *  - d_rgb8: optional, n_frames band buffers of RGB8 = Color::as_u8 (color.rs:43-46) of each
 *            pixel, written by the render's last pass (no separate quantise launch) -- 3 B per
 *            pixel for the multi-GPU gather instead of 12.
 * A queue overflow cannot be returned by a stream-ordered call: it is latched in the scene
 * and reported by rt_scene_sync_status.
 * HOST WAIT (every *_async render, rt_render_frame_async and the multi-device shares): a pass
 * with more level-0 items (pixels x frames x samples of this rank) or a greater depth than any
 * pass this handle has completed is checked before the call returns -- the call waits for
 * `stream` and the handle's other streams, and if a ray queue overflowed it grows the node
 * pool and renders the pass again (up to 8 times).  Passes no larger than a checked one are
 * enqueued without any host wait.  So the first pass of a new size blocks; render one such
 * pass before capturing a stream into a graph: while `stream` is being captured, a pass that
 * would need the check returns RT_ERR_UNSUPPORTED and enqueues nothing.  Tuning key
 * node_cap pins the pool and skips the check (an overflow is then only latched). */
rt_status rt_render_bands_ex_async(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames, uint32_t depth,
                                   uint32_t spp, uint32_t seed, uint32_t band_rows, uint32_t rank, uint32_t world,
                                   float* d_rgb, uint8_t* d_rgb8, uint64_t* d_counters, void* stream);

/* A frame batch (as rt_render_bands_batch_async) whose pixels land in place: d_frames holds
 * n_frames WHOLE row-major frames (y_res x x_res x 3 floats each; d_frames8 optional, the
 * Color::as_u8 bytes, same layout), and this call writes only this rank's rows of them --
 * no band buffer, no padding rows, no un-permute.  `world` band shares of one device (each
 * its own scene handle and stream) fill the same frames side by side; a pass then mixes
 * twice (world 2) the frames of a whole-frame pass of the same size.  spp == 1 only.
 * Every pixel equals rt_render's bit for bit.  No reference counterpart: the throughput
 * form of render() (src/render.rs:31) over frames. */
rt_status rt_render_bands_direct_async(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames,
                                       uint32_t depth, uint32_t band_rows, uint32_t rank, uint32_t world,
                                       float* d_frames, uint8_t* d_frames8, uint64_t* d_counters, void* stream);

/* Waits for every stream-ordered render enqueued on `scene` so far, on every stream one ran
 * on (the scene records an event per such stream after each render), and reports whether
 * one of them overflowed a ray queue: RT_ERR_CAPACITY (that frame is incomplete; the flag is
 * then cleared, and the next pass on this scene gets a node pool twice as large) or RT_OK.
 * rt_render / rt_render_spp never need it: they grow the pool and render again. */
rt_status rt_scene_sync_status(rt_scene* scene);

/* Stochastic supersampling (BASELINE config 5; the reference has no equivalent, SURVEY.md
 * §7 step 6).  Sample k (0 <= k < spp) of pixel (u, v) is Camera::get_ray's ray through
 * (u + jx, v + jy) -- x = x_min + ((float)u + jx) * x_delta, y = y_max - ((float)v + jy) *
 * y_delta (render.rs:178-185 with the jitter added) -- where, with pixel = v * x_res + u
 * and mix32 the 32-bit finaliser x ^= x>>16; x *= 0x7feb352d; x ^= x>>15;
 * x *= 0x846ca68b; x ^= x>>16:
 *     h  = mix32(mix32(seed ^ 0x9e3779b9) ^ pixel)
 *     j_dim = (mix32(h ^ mix32(2k + dim + 1)) >> 8) * 2^-24     (dim 0: jx, 1: jy)
 * The pixel is the f32 sum of its sample colours in sample order (sample 0 first),
 * divided by (float)spp.  spp == 1 is rt_render exactly (no jitter).  The counters count
 * pixel samples. */
rt_status rt_render_spp(const rt_scene* scene, const rt_camera* camera, uint32_t depth,
                        uint32_t spp, uint32_t seed, const rt_render_opts* opts,
                        float* rgb, uint8_t* rgb8);
rt_status rt_render_bands_spp_async(const rt_scene* scene, const rt_camera* camera,
                                    uint32_t depth, uint32_t spp, uint32_t seed,
                                    uint32_t band_rows, uint32_t rank, uint32_t world,
                                    float* d_rgb, uint64_t* d_counters, void* stream);

/* Number of rows (including padding) a rank's band buffer holds. */
uint32_t rt_band_rows_per_rank(uint32_t y_res, uint32_t band_rows, uint32_t world);

/* Scatter the `world` gathered band buffers (rank-major: world * rows_per_rank rows of
 * x_res*3 floats) into a row-major frame `d_frame` (y_res rows), on `stream`. */
rt_status rt_unpermute_bands_async(const float* d_gathered, uint32_t x_res, uint32_t y_res,
                                   uint32_t band_rows, uint32_t world, float* d_frame,
                                   void* stream);

/* rt_unpermute_bands_async for RGB8 band buffers (rt_render_bands_ex_async's d_rgb8). */
rt_status rt_unpermute_bands_u8_async(const uint8_t* d_gathered, uint32_t x_res, uint32_t y_res,
                                      uint32_t band_rows, uint32_t world, uint8_t* d_frame, void* stream);

/* A gathered frame batch in one launch: d_gathered holds, per rank, stride_frames band
 * buffers of which the first n_frames are filled (rank-major: rank r's buffer of frame f
 * is the (r * stride_frames + f)-th buffer of rt_band_rows_per_rank rows) -- what one
 * gather of every rank's rt_render_bands_batch_async output gives; frame f lands at
 * d_frames + f * y_res * x_res * 3. */
rt_status rt_unpermute_bands_batch_async(const float* d_gathered, uint32_t x_res, uint32_t y_res,
                                         uint32_t band_rows, uint32_t world, uint32_t n_frames,
                                         uint32_t stride_frames, float* d_frames, void* stream);
rt_status rt_unpermute_bands_batch_u8_async(const uint8_t* d_gathered, uint32_t x_res, uint32_t y_res,
                                            uint32_t band_rows, uint32_t world, uint32_t n_frames,
                                            uint32_t stride_frames, uint8_t* d_frames, void* stream);

/* Saves a row-major RGB8 frame (Color::as_u8 values) as PNG, BMP or PPM, chosen by the
 * file extension (.png default) -- bmp.rs:8-19 / main.rs:71-74 (host code). */
rt_status rt_write_image(const char* path, const uint8_t* rgb8, uint32_t x_res, uint32_t y_res);

/* Color::as_u8 (color.rs:43-46) of a row-major float frame, on the device. */
rt_status rt_quantize_u8_async(const float* d_rgb, size_t n_values, uint8_t* d_rgb8,
                               void* stream);

/* Algorithmic f32 operation count of one scene scan:
 * sphere 57, triangle 52, cube 33 + 12*52, plane 49 per ray-primitive test. */
uint64_t rt_scene_flops_per_scan(const rt_scene* scene);

/* Bytes of the flattened device scene (for the HBM-traffic accounting). */
uint64_t rt_scene_device_bytes(const rt_scene* scene);

/* Lane-weighted counts of the ray-primitive and ray-box tests the scene's scans ran
 * since the last reset, in this order: child-box pairs, diagonal-sphere pairs, general
 * spheres, triangle pairs, cube boxes, full cubes (12 triangles), grazing cone tests
 * (blocks of 8 triangles), planes, grazing normal tests (blocks of 8); then shader-clock
 * cycles per wave in child-box tests, leaf tests, the grazing pass and whole scans, and
 * in the trace kernel's ray fetch, post-scan work and own-shape shadow tests.
 * Synchronises the device; reset != 0 zeroes the counts after reading.  `out` may be
 * NULL. */
#define RT_SCAN_OPS_N 16
rt_status rt_scene_scan_ops(rt_scene* scene, uint64_t* out, uint32_t n, int32_t reset);

/* Counting is instrumentation: renders after rt_scene_set_scan_counting(scene, 1) run
 * the counting variants of the level-synchronous kernels; the default (0) runs uncounted
 * kernels.  Frames are identical.  (bench.py's roofline: one untimed counting frame.) */
rt_status rt_scene_set_scan_counting(rt_scene* scene, int32_t enable);

/* Frames in flight: the share (percent, 1..100, default 100) of a full chip that one
 * render pass's persistent trace grids take.  Several passes on several streams then run
 * side by side instead of one filling every CU slot until its level is drained (bench /
 * FramePipeline: 75 with 4 passes in flight).  Results do not change. */
rt_status rt_scene_set_grid_share(rt_scene* scene, int32_t percent);

/* 1 if the scene's scans walk the culling hierarchy (the default; tuning "bvh=0" at
 * creation turns it off), 0 if they test every shape. */
int32_t rt_scene_uses_bvh(const rt_scene* scene);

/* Per-kernel device time of this handle's own render passes (not its band shares' or
 * devices'): with timing on, every launch group of a pass -- a trace level, a task-queue sort,
 * the shadow-queue sort, the shadow pass, a combine level -- is bracketed by HIP events on the
 * pass's stream.  One pass at a time on one stream gives each kind's exclusive time
 * (bench.py's per-kernel roofline).  rt_scene_kernel_times waits for the recorded events and
 * writes ms[kind] summed over the passes since the last reset (RT_KT_* below; ms[RT_KT_LAUNCHES]
 * = the number of spans); reset != 0 forgets them.  Measurement only: the events cost time. */
enum { RT_KT_TRACE = 0, RT_KT_SORT_TASKS = 1, RT_KT_SORT_SHADOW = 2, RT_KT_SHADOW = 3, RT_KT_COMBINE = 4,
       RT_KT_LAUNCHES = 5 };
rt_status rt_scene_set_kernel_timing(rt_scene* scene, int32_t enable);
rt_status rt_scene_kernel_times(rt_scene* scene, float* ms, uint32_t n, int32_t reset);

/* ---- ray forest (src/render_tree.rs) -------------------------------------------------
 * generate_ray_forest(camera, scene, w, h, depth) -> RayForest (render_tree.rs:147-164):
 * traces every pixel's ray tree (the same rays, shadow tests and child rules as
 * render.rs) once and keeps every intersection on the device. */
typedef struct rt_forest rt_forest;
rt_status rt_forest_create(rt_scene* scene, const rt_camera* camera, uint32_t depth, rt_forest** out);
/* A forest uses its scene's stream and materials: destroy it before its scene. */
rt_status rt_forest_destroy(rt_forest* forest);

/* render_forest(&forest, &mut buffer, ambient) (render_tree.rs:121-127, render_ray_tree
 * :214-255): shades every tree with the scene's CURRENT materials into `rgb`
 * (row-major y_res x x_res x 3 floats).  Note the forest's shading differs from
 * render.rs: the reflected term uses the hit's eye_dir as light direction, the refracted
 * term is not scaled by the diffuse colour. */
rt_status rt_forest_render(rt_forest* forest, float* rgb);

/* render_forest_filter(&forest, &mut buffer, ambient, mutated_shapes)
 * (render_tree.rs:129-145): re-shades only the pixels whose tree holds one of
 * `mutated_ids`; the other pixels of `rgb` are left as they are.  Shape ids are the
 * reference's: the insertion index, except that a cube hit reports the id of the cube's
 * inner triangle (0..11, cube.rs:93-99). */
rt_status rt_forest_render_filter(rt_forest* forest, const int32_t* mutated_ids, uint32_t n_ids, float* rgb);

/* RayTree::size per pixel (render_tree.rs:39-48, row-major), for RayForest::stats (:73-93). */
rt_status rt_forest_tree_sizes(rt_forest* forest, uint32_t* sizes);

/* RayForest::trees_with(shape_id) (render_tree.rs:66-71). */
rt_status rt_forest_trees_with(rt_forest* forest, int32_t shape_id, uint64_t* count);

/* Ray counts of the build (node rays, shadow rays, pixels). */
rt_status rt_forest_counters(const rt_forest* forest, rt_counters* out);

/* Device time (HIP events, ms) of the build's trace + shadow passes (its last attempt) and of
 * the last rt_forest_render / _render_filter (the mark and shade kernels; host copies
 * excluded; 0 before the first shade).  Either pointer may be NULL. */
rt_status rt_forest_timings(const rt_forest* forest, float* build_ms, float* shade_ms);

/* Replace material `index`'s parameters (same kind) -- the GUI's material edits
 * (gui.rs:221-236).  Affects later renders and forest shades. */
rt_status rt_scene_set_material(rt_scene* scene, uint32_t index, const rt_material* material);

/* Brings a handle up to date with `desc` -- the caller's Scene as it is now -- so that a
 * render() binding can keep ONE handle across calls (render.rs:31 takes the same &Scene every
 * frame: main.rs:137-140, 244-261) instead of rebuilding the device scene per call:
 *  - `desc` equal to the description the handle renders (byte for byte): nothing; *what = 0;
 *  - only materials differ, each keeping its kind: rt_scene_set_material per edited index
 *    (no rebuild); *what = 1;
 *  - anything else (a shape added or transformed, a light, the ambient, a material's kind or
 *    count): the scene is rebuilt with the handle's device and tuning and adopted in place --
 *    the handle, its stream, workspace, band shares and devices stay valid; *what = 2.
 * Renders on the handle must not run concurrently with it; it waits for the handle's streams.
 * A stream-ordered render's unreported status (rt_scene_sync_status) is returned first and
 * the update is then not made.  A forest created before a rebuild (*what = 2) keeps its trees
 * (rt_forest_tree_sizes / _trees_with / _counters still answer for them) but can no longer be
 * shaded: rt_forest_render / _render_filter return RT_ERR_INVALID_ARG -- its nodes hold the old
 * scene's material indices and light count; create a new forest.  Material edits in place
 * (*what = 1) keep forests valid and are seen by their next shade.  Every edited material is
 * validated before the first is applied.  `what` may be NULL.  Errors of the rebuild (e.g. RT_ERR_SINGULAR_MATRIX) leave the handle
 * rendering its previous scene. */
rt_status rt_scene_update(rt_scene* scene, const rt_scene_desc* desc, int32_t* what);

const char* rt_status_str(rt_status status);
int32_t rt_api_version(void);
/* The most frames one pipeline pass takes (rt_render_bands_batch_async's n_frames). */
uint32_t rt_max_frames(void);

#ifdef __cplusplus
}
#endif

#endif /* RT_API_H */
