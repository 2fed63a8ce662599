// rt_internal.hpp -- what rt_multi.cpp (the multi-device render behind rt_scene_create_multi)
// needs from rt_scene.cpp's scene handle.  Not part of the C ABI.
#pragma once
#include <functional>

#include <hip/hip_runtime.h>

#include "../../include/rt_api.h"
#include "rt_tune.hpp"

struct rt_multi_state;

// The multi-device state a primary scene handle carries (null: a one-device scene).
rt_multi_state*& rt_scene_multi(rt_scene* s);
int rt_scene_device_of(const rt_scene* s);
// The handle's tuning (rt_tune.hpp).
const Tune& rt_scene_tune(const rt_scene* s);

// rt_render_spp on a multi-device scene (rt_multi.cpp).
rt_status rt_multi_render(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                          const rt_render_opts* opts, float* rgb, uint8_t* rgb8);
rt_status rt_multi_render_state(rt_multi_state* m, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                                const rt_render_opts* opts, float* rgb, uint8_t* rgb8);
// A multi-device state around the primary handle s0 (not owned): clones of s0 on
// devices[1..], a stream per rank; RCCL when the devices are distinct and allow_rccl.
rt_status rt_multi_build(rt_scene* s0, const int32_t* devices, uint32_t n_devices, bool allow_rccl,
                         rt_multi_state** out);
void rt_multi_set_band_rows(rt_multi_state* m, uint32_t band_rows);
// Applies `f` to every clone (devices[1..]) of a multi-device scene; first error wins.
rt_status rt_multi_each(rt_multi_state* m, const std::function<rt_status(rt_scene*)>& f);
// the last render's per-rank finish times (ms after its start) on one device's copy
// exchange; RT_ERR_UNSUPPORTED when it did not run that way
rt_status rt_multi_share_ms(rt_multi_state* m, float* ms, uint32_t n);
// ... and each rank's copy-out time (from its finish to its band in the caller's buffers)
rt_status rt_multi_copy_ms(rt_multi_state* m, float* ms, uint32_t n);
void rt_multi_free(rt_multi_state* m);
// Every rank of a multi-device state, ranks[0] included.
rt_status rt_multi_each_rank(rt_multi_state* m, const std::function<rt_status(rt_scene*)>& f);
// rt_render_frame_async's two band shares on one device (rt_multi.cpp): share 0 = rows
// [0, rows) straight into d_rgb, share 1 = rows [rows, y_res) through its band buffer;
// fork from and join back into `stream`.  y_res / 2 <= rows < y_res.
rt_status rt_multi_render_frame_async(rt_multi_state* m, const rt_camera* cam, uint32_t depth, uint32_t rows,
                                      float* d_rgb, uint8_t* d_rgb8, uint64_t* d_counters, hipStream_t stream);
// the previous rt_multi_render_frame_async's share spans once complete (never waits)
rt_status rt_multi_async_share_ms(rt_multi_state* m, float* ms, uint32_t n);
// rt_scene_sync_status of this handle's own workspace only (not its split shares)
extern "C" rt_status rt_scene_sync_own(rt_scene* s);
