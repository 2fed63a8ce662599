// rt_internal.hpp -- what rt_multi.cpp (the multi-device render behind rt_scene_create_multi)
// needs from rt_api.cpp's scene handle.  Not part of the C ABI.
#pragma once
#include <functional>

#include "../../include/rt_api.h"

struct rt_multi_state;

// The multi-device state a primary scene handle carries (null: a one-device scene).
rt_multi_state*& rt_scene_multi(rt_scene* s);
int rt_scene_device_of(const rt_scene* s);

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
