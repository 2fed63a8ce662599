// scene.hpp -- C++ host mirror of the reference's Scene / Camera / RenderBuffer API.
//
// The reference builds scenes through src/scene/mod.rs (Scene::add_shape, add_light,
// set_ambient), src/scene/{sphere,plane,triangle,cube,material}.rs constructors and
// src/math (Matrix::translate/scale/rotate_*, `*`), then calls
// render::render(&camera, &scene, &mut buffer, depth) (src/render.rs:31).  This header
// keeps those names and argument meanings so src/my_scene.rs reads the same in C++
// (host/my_scene.cpp); `render()` flattens the scene into an rt_scene_desc and crosses
// the C ABI (include/rt_api.h) into the HIP megakernel.
//
// Differences forced by the boundary:
//  * TexturePhong takes Texture programs (a closed enum) instead of fn pointers
//    (material.rs:3); checkerboard/dim_white of my_scene.rs are provided.
//  * Errors are rt_status codes, not panics.
#pragma once

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/rt_api.h"
#include "../../../include/rt_scenes.h"

namespace rust_tracer {

struct Vector3 {
    float x = 0, y = 0, z = 0;
    Vector3() = default;
    Vector3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
};

struct Point3 {
    float x = 0, y = 0, z = 0;
    Point3() = default;
    Point3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
};

// Row-major 4x4 (src/math/matrix.rs).  Products accumulate left to right from 0.,
// exactly as Matrix::mat_mul does (matrix.rs:68-86).
struct Matrix {
    float m[4][4];
    static Matrix identity();
    static Matrix scale(float x, float y, float z);       // matrix.rs:155-164
    static Matrix translate(float x, float y, float z);   // matrix.rs:166-175
    static Matrix rotate_x(float degrees);                // matrix.rs:177-189
    static Matrix rotate_y(float degrees);                // matrix.rs:191-203
    static Matrix rotate_z(float degrees);                // matrix.rs:205-217
    Matrix operator*(const Matrix& rhs) const;
};

struct Color {
    float r = 0, g = 0, b = 0;
    Color() = default;
    Color(float r_, float g_, float b_) : r(r_), g(g_), b(b_) {}
};
inline Color operator*(float s, const Color& c) { return Color(s * c.r, s * c.g, s * c.b); }

namespace colors {  // color.rs:8-38
const Color BLACK(0.f, 0.f, 0.f);
const Color WHITE(1.f, 1.f, 1.f);
const Color RED(1.f, 0.f, 0.f);
const Color GREEN(0.f, 1.f, 0.f);
const Color BLUE(0.f, 0.f, 1.f);
}  // namespace colors

// A texture program: the GPU-evaluable replacement for `ColorFun`.
struct Texture {
    int32_t kind = RT_TEX_CONST;
    Color color;
    static Texture constant(const Color& c) { Texture t; t.color = c; return t; }
    static Texture checkerboard() { Texture t; t.kind = RT_TEX_CHECKERBOARD; return t; }
};

struct Material {  // Phong (material.rs:24-52) and TexturePhong (material.rs:103-130)
    int32_t kind = RT_MAT_PHONG;
    Texture ambient, diffuse, specular;
    float power = 0, reflectivity = 0, refraction_index = 0;
};
using MaterialRef = std::shared_ptr<Material>;  // Rc<RefCell<dyn Material>>

MaterialRef Phong(const Color& ambient, const Color& diffuse, const Color& specular, float power,
                  float reflectivity, float refraction_index);
MaterialRef TexturePhong(const Texture& ambient, const Texture& diffuse, const Texture& specular,
                         float power, float reflectivity, float refraction_index);

// Renderables.  Geometry is kept as the reference's constructors receive it; the
// preprocessing (inverse, plane axes, triangle normal, cube triangles) happens in the
// library at rt_scene_create.
struct Shape {
    int32_t kind = RT_SHAPE_SPHERE;
    int32_t id = 0;  // set by Scene::add_shape (mod.rs:40-44)
    MaterialRef material;
    Matrix transform = Matrix::identity();
    float data[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    std::string name;
    void set_transform(const Matrix& m) { transform = m; }  // e.g. sphere.rs:100-103
};
Shape Sphere(MaterialRef material);                                    // sphere.rs:20-28
Shape SphereWithName(const std::string& name, MaterialRef material);  // sphere.rs:30-38
Shape Plane(const Point3& origin, const Vector3& normal, MaterialRef material);  // plane.rs:22
Shape Triangle(const Point3& v0, const Point3& v1, const Point3& v2, MaterialRef material);
Shape Cube(MaterialRef material);                                      // cube.rs:21-77

struct Light {
    int32_t kind = RT_LIGHT_POINT;
    Point3 pos;
    Color color;
};
Light PointLight(const Point3& pos, const Color& color);  // mod.rs:183-187
Light AmbientLight(const Color& color);                   // mod.rs:228-233

class Scene {  // mod.rs:22-85
public:
    Scene();
    ~Scene();
    Scene(const Scene& o);             // the copy renders through a device scene of its own
    Scene& operator=(const Scene& o);
    Scene(Scene&&) noexcept;
    Scene& operator=(Scene&&) noexcept;

    void add_shape(Shape s);
    void add_light(const Light& l) { lights_.push_back(l); }
    void set_ambient(const Color& c) { ambient_ = c; }
    const Color& ambient() const { return ambient_; }
    const std::vector<Shape>& shapes() const { return shapes_; }
    const std::vector<Light>& lights() const { return lights_; }
    const Shape* find_shape(const std::string& name) const;
    Shape* find_shape_mut(const std::string& name);  // mod.rs:66-74 (e.g. set_transform after add)
    // Renderable::size (mod.rs:124-126): a cube counts its 12 triangles (cube.rs:113-115)
    size_t size() const;

    // Flatten into the C-ABI description (materials de-duplicated by identity, shapes and
    // lights in insertion order).  The returned holder owns every array it points at.
    struct Flat {
        std::vector<rt_material> materials;
        std::vector<rt_shape> shapes;
        std::vector<rt_light> lights;
        rt_scene_desc desc;
    };
    std::unique_ptr<Flat> flatten() const;

    // The device scene render() keeps across calls (the reference's render() takes the same
    // &Scene every frame, main.rs:137-140): created by the first render(), brought up to date
    // by rt_scene_update on later ones -- nothing to do when the scene is unchanged, material
    // edits in place (Rc<RefCell<Material>> edits through a MaterialRef land here too), a
    // rebuild after any other edit.  Freed with the Scene.
    struct DeviceCache;
    DeviceCache& device_cache() const;

private:
    Color ambient_ = colors::BLACK;
    std::vector<Shape> shapes_;
    std::vector<Light> lights_;
    mutable std::unique_ptr<DeviceCache> cache_;  // (a moved-from Scene gets a new one when rendered)
    mutable std::mutex cache_init_;
};

struct Camera {  // render.rs:155-176
    Point3 origin{0.f, 0.f, -8.f};
    float x_min = -3.f, x_max = 3.f, y_min = -3.f, y_max = 3.f;
    uint32_t x_res = 0, y_res = 0;
    Camera(uint32_t xr, uint32_t yr) : x_res(xr), y_res(yr) {}
    rt_camera to_c() const;
};

struct RenderBuffer {  // render.rs:5-19; stored row-major [v][u] (the reference is [u][v])
    uint32_t w = 0, h = 0;
    std::vector<Color> buf;
    RenderBuffer(uint32_t w_, uint32_t h_) : w(w_), h(h_), buf((size_t)w_ * h_) {}
    Color& at(uint32_t u, uint32_t v) { return buf[(size_t)v * w + u]; }
    const Color& at(uint32_t u, uint32_t v) const { return buf[(size_t)v * w + u]; }
};

// render.rs:31-38 through the C ABI.  `device` = -1 uses the current HIP device.  The scene's
// device handle is kept across calls (Scene::DeviceCache); `update` (optional) reports what
// this call did to it: -1 created, 0 reused as is, 1 materials edited in place, 2 rebuilt.
rt_status render(const Camera& camera, const Scene& scene, RenderBuffer& buffer, uint32_t depth,
                 int32_t device = -1, rt_counters* counters = nullptr, float* kernel_ms = nullptr,
                 int32_t* update = nullptr);

// my_scene.rs:45-120
void create_scene(Scene& scene);
// render.rs:233-249
void create_bench_128_scene(Scene& scene);
// SURVEY.md §8(d) synthetic scene
void create_synth_scene(Scene& scene, const rt_synth_params& p);

}  // namespace rust_tracer
