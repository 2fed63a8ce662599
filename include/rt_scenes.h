/*
 * rt_scenes.h -- scene descriptions built by the C++ host mirror of the reference's
 * Scene API (rust_tracer_amd/csrc/host).  These are callers of the boundary, not part
 * of it: the reference builds the same scenes in Rust (src/my_scene.rs:45-120,
 * src/render.rs:233-249) before calling render().
 *
 * Descriptions returned here are owned by the library; release them with rt_desc_free.
 */
#ifndef RT_SCENES_H
#define RT_SCENES_H

#include "rt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* my_scene.rs:45-120: 3 spheres, 2 checkerboard planes, 1 glass cube, 3 point lights. */
rt_status rt_desc_my_scene(rt_scene_desc** out);

/* render.rs:233-249 (`render_128x128` bench): one Phong(WHITE,RED,WHITE,60,1,0) sphere
 * scaled (1, 2.25, 1), no lights, ambient BLACK. */
rt_status rt_desc_bench_128(rt_scene_desc** out);

/* The seeded synthetic scene of SURVEY.md §8(d): my_scene's two textured planes, its
 * three lights and ambient 0.1, plus n_spheres spheres (radius U[r_min, r_max]),
 * n_cubes cubes and n_triangles loose triangles, all drawn from splitmix64(seed). */
typedef struct rt_synth_params {
    uint64_t seed;
    uint32_t n_spheres;
    uint32_t n_cubes;
    uint32_t n_triangles;
    float r_min, r_max;
} rt_synth_params;
rt_status rt_desc_synth(const rt_synth_params* params, rt_scene_desc** out);

/* BASELINE.json configs: 2 -> synth(seed 1, 100 spheres, r U[0.15,0.45]);
 * 3, 4, 5 -> synth(seed 2, 600 spheres r U[0.06,0.2], 25 cubes, 100 triangles). */
rt_status rt_synth_config(int32_t config, rt_synth_params* out);

void rt_desc_free(rt_scene_desc* desc);

/* The C++ host mirror's render() (csrc/host/scene.hpp; render.rs:31-38) called n_calls times
 * on ONE Scene into one RenderBuffer -- the reference's bench loop (main.rs:137-140,
 * render_scene_basic main.rs:244-261) through the drop-in seam, whose Scene keeps its device
 * scene across calls.  scene: 0 = my_scene.rs, 2 .. 5 = rt_synth_config(scene).  edit,
 * applied before the last call (n_calls >= 2): 0 none; 1 set_transform of the first sphere
 * (find_shape_mut, translated 0.1 in x); 2 the first shape's material's diffuse colour set to
 * (0.25, 0.5, 0.75) (an Rc<RefCell<Material>> edit); 3 a point light added.  Out: ms[i] = wall time of call i
 * (the frame's device-to-host copy included), updates[i] = what render() did to the device
 * scene (-1 created, 0 reused, 1 materials edited in place, 2 rebuilt); rgb (optional,
 * x_res * y_res * 3 floats) = the last call's frame; rgb_fresh (optional) = the same edited
 * Scene rendered by a newly created handle, for comparison.  Test and bench harness. */
rt_status rt_mirror_render_calls(int32_t scene, uint32_t x_res, uint32_t y_res, uint32_t depth, uint32_t n_calls,
                                 int32_t edit, int32_t device, float* ms, int32_t* updates, float* rgb,
                                 float* rgb_fresh);

#ifdef __cplusplus
}
#endif
#endif
