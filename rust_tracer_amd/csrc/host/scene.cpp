// scene.cpp -- host mirror of the reference Scene API (see scene.hpp) and the scene
// builders exported through include/rt_scenes.h.
#include "scene.hpp"

#include <chrono>
#include <cmath>
#include <cstring>
#include <map>

#include "../../../include/rt_scenes.h"

namespace rust_tracer {

static const float PI_F = 3.14159265358979323846f;  // std::f32::consts::PI

Matrix Matrix::identity() {
    Matrix r;
    std::memset(r.m, 0, sizeof(r.m));
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.f;
    return r;
}
Matrix Matrix::scale(float x, float y, float z) {
    Matrix r = identity();
    r.m[0][0] = x;
    r.m[1][1] = y;
    r.m[2][2] = z;
    return r;
}
Matrix Matrix::translate(float x, float y, float z) {
    Matrix r = identity();
    r.m[0][3] = x;
    r.m[1][3] = y;
    r.m[2][3] = z;
    return r;
}
// Angles arrive in degrees and become radians as (angle / 180) * PI in f32.  The
// reference's rustc release build constant-folds cos/sin of those constants in
// double and rounds to f32; we do the same at run time so host matrices match.
static void cos_sin(float degrees, float& c, float& s) {
    float rads = degrees / 180.0f * PI_F;
    c = (float)std::cos((double)rads);
    s = (float)std::sin((double)rads);
}
Matrix Matrix::rotate_x(float d) {
    float c, s;
    cos_sin(d, c, s);
    Matrix r = identity();
    r.m[1][1] = c; r.m[1][2] = -s;
    r.m[2][1] = s; r.m[2][2] = c;
    return r;
}
Matrix Matrix::rotate_y(float d) {
    float c, s;
    cos_sin(d, c, s);
    Matrix r = identity();
    r.m[0][0] = c; r.m[0][2] = s;
    r.m[2][0] = -s; r.m[2][2] = c;
    return r;
}
Matrix Matrix::rotate_z(float d) {
    float c, s;
    cos_sin(d, c, s);
    Matrix r = identity();
    r.m[0][0] = c; r.m[0][1] = -s;
    r.m[1][0] = s; r.m[1][1] = c;
    return r;
}
Matrix Matrix::operator*(const Matrix& a) const {
    Matrix r;
    for (int row = 0; row < 4; row++)
        for (int col = 0; col < 4; col++) {
            float sum = 0.f;
            for (int k = 0; k < 4; k++) sum += m[row][k] * a.m[k][col];
            r.m[row][col] = sum;
        }
    return r;
}

MaterialRef Phong(const Color& a, const Color& d, const Color& s, float power, float refl, float ri) {
    auto m = std::make_shared<Material>();
    m->kind = RT_MAT_PHONG;
    m->ambient = Texture::constant(a);
    m->diffuse = Texture::constant(d);
    m->specular = Texture::constant(s);
    m->power = power;
    m->reflectivity = refl;
    m->refraction_index = ri;
    return m;
}

MaterialRef TexturePhong(const Texture& a, const Texture& d, const Texture& s, float power,
                         float refl, float ri) {
    auto m = std::make_shared<Material>();
    m->kind = RT_MAT_TEXTURE_PHONG;
    m->ambient = a;
    m->diffuse = d;
    m->specular = s;
    m->power = power;
    m->reflectivity = refl;
    m->refraction_index = ri;
    return m;
}

Shape Sphere(MaterialRef material) {
    Shape s;
    s.kind = RT_SHAPE_SPHERE;
    s.material = material;
    s.name = "Sphere";
    return s;
}
Shape SphereWithName(const std::string& name, MaterialRef material) {
    Shape s = Sphere(material);
    s.name = name;
    return s;
}
Shape Plane(const Point3& o, const Vector3& n, MaterialRef material) {
    Shape s;
    s.kind = RT_SHAPE_PLANE;
    s.material = material;
    s.name = "Plane";
    const float d[6] = {o.x, o.y, o.z, n.x, n.y, n.z};
    std::memcpy(s.data, d, sizeof(d));
    return s;
}
Shape Triangle(const Point3& a, const Point3& b, const Point3& c, MaterialRef material) {
    Shape s;
    s.kind = RT_SHAPE_TRIANGLE;
    s.material = material;
    s.name = "Triable";  // triangle.rs:113-115
    const float d[9] = {a.x, a.y, a.z, b.x, b.y, b.z, c.x, c.y, c.z};
    std::memcpy(s.data, d, sizeof(d));
    return s;
}
Shape Cube(MaterialRef material) {
    Shape s;
    s.kind = RT_SHAPE_CUBE;
    s.material = material;
    s.name = "Cube";
    return s;
}

Light PointLight(const Point3& pos, const Color& color) {
    Light l;
    l.kind = RT_LIGHT_POINT;
    l.pos = pos;
    l.color = color;
    return l;
}
Light AmbientLight(const Color& color) {
    Light l;
    l.kind = RT_LIGHT_AMBIENT;
    l.color = color;
    return l;
}

struct Scene::DeviceCache {
    std::mutex m;
    rt_scene* handle = nullptr;
    int32_t device = -1;
    ~DeviceCache() {
        if (handle) rt_scene_destroy(handle);
    }
};

Scene::Scene() : cache_(new DeviceCache()) {}
Scene::~Scene() = default;
Scene::Scene(const Scene& o)
    : ambient_(o.ambient_), shapes_(o.shapes_), lights_(o.lights_), cache_(new DeviceCache()) {}
Scene& Scene::operator=(const Scene& o) {
    if (this != &o) {
        ambient_ = o.ambient_;
        shapes_ = o.shapes_;
        lights_ = o.lights_;  // the device handle stays; the next render() updates it
    }
    return *this;
}
Scene::Scene(Scene&& o) noexcept
    : ambient_(o.ambient_), shapes_(std::move(o.shapes_)), lights_(std::move(o.lights_)), cache_(std::move(o.cache_)) {}
Scene& Scene::operator=(Scene&& o) noexcept {
    if (this != &o) {
        ambient_ = o.ambient_;
        shapes_ = std::move(o.shapes_);
        lights_ = std::move(o.lights_);
        cache_ = std::move(o.cache_);
    }
    return *this;
}
Scene::DeviceCache& Scene::device_cache() const {
    std::lock_guard<std::mutex> lock(cache_init_);
    if (!cache_) cache_.reset(new DeviceCache());
    return *cache_;
}

Shape* Scene::find_shape_mut(const std::string& name) {
    for (auto& s : shapes_)
        if (s.name == name) return &s;
    return nullptr;
}

void Scene::add_shape(Shape s) {
    s.id = (int32_t)shapes_.size();
    shapes_.push_back(std::move(s));
}

size_t Scene::size() const {
    size_t n = 0;
    for (const Shape& s : shapes_) n += s.kind == RT_SHAPE_CUBE ? 12u : 1u;
    return n;
}

const Shape* Scene::find_shape(const std::string& name) const {
    for (const auto& s : shapes_)
        if (s.name == name) return &s;
    return nullptr;
}

static rt_color cc(const Color& c) { return rt_color{c.r, c.g, c.b}; }
static rt_texture ct(const Texture& t) { return rt_texture{t.kind, cc(t.color)}; }

std::unique_ptr<Scene::Flat> Scene::flatten() const {
    std::unique_ptr<Flat> f(new Flat());
    std::map<const Material*, int32_t> index;
    for (const auto& s : shapes_) {
        const Material* m = s.material.get();
        if (!m) continue;
        if (index.count(m)) continue;
        index[m] = (int32_t)f->materials.size();
        rt_material r;
        std::memset(&r, 0, sizeof(r));
        r.kind = m->kind;
        r.ambient = ct(m->ambient);
        r.diffuse = ct(m->diffuse);
        r.specular = ct(m->specular);
        r.power = m->power;
        r.reflectivity = m->reflectivity;
        r.refraction_index = m->refraction_index;
        f->materials.push_back(r);
    }
    for (const auto& s : shapes_) {
        rt_shape r;
        std::memset(&r, 0, sizeof(r));
        r.kind = s.kind;
        r.material = s.material ? index[s.material.get()] : -1;
        std::memcpy(r.transform, s.transform.m, sizeof(r.transform));
        std::memcpy(r.data, s.data, sizeof(r.data));
        f->shapes.push_back(r);
    }
    for (const auto& l : lights_) {
        rt_light r;
        std::memset(&r, 0, sizeof(r));
        r.kind = l.kind;
        r.pos[0] = l.pos.x; r.pos[1] = l.pos.y; r.pos[2] = l.pos.z;
        r.color = cc(l.color);
        f->lights.push_back(r);
    }
    f->desc.n_materials = (uint32_t)f->materials.size();
    f->desc.materials = f->materials.data();
    f->desc.n_shapes = (uint32_t)f->shapes.size();
    f->desc.shapes = f->shapes.data();
    f->desc.n_lights = (uint32_t)f->lights.size();
    f->desc.lights = f->lights.data();
    f->desc.ambient = cc(ambient_);
    return f;
}

rt_camera Camera::to_c() const {
    rt_camera c;
    c.origin[0] = origin.x; c.origin[1] = origin.y; c.origin[2] = origin.z;
    c.x_min = x_min; c.x_max = x_max; c.y_min = y_min; c.y_max = y_max;
    c.x_res = x_res; c.y_res = y_res;
    return c;
}

rt_status render(const Camera& camera, const Scene& scene, RenderBuffer& buffer, uint32_t depth,
                 int32_t device, rt_counters* counters, float* kernel_ms, int32_t* update) {
    if (buffer.w != camera.x_res || buffer.h != camera.y_res) return RT_ERR_INVALID_ARG;
    auto flat = scene.flatten();
    Scene::DeviceCache& c = scene.device_cache();
    std::lock_guard<std::mutex> lock(c.m);  // one render of a Scene at a time (the handle is !Sync)
    if (c.handle && c.device != device) {
        rt_scene_destroy(c.handle);
        c.handle = nullptr;
    }
    rt_status st = RT_OK;
    if (!c.handle) {
        st = rt_scene_create(&flat->desc, device, &c.handle);
        if (st != RT_OK) {
            c.handle = nullptr;
            return st;
        }
        c.device = device;
        if (update) *update = -1;
    } else {
        int32_t what = 0;
        st = rt_scene_update(c.handle, &flat->desc, &what);
        if (st != RT_OK) return st;
        if (update) *update = what;
    }
    rt_camera cam = camera.to_c();
    rt_render_opts opts;
    opts.device = device;
    opts.counters = counters;
    opts.kernel_ms = kernel_ms;
    static_assert(sizeof(Color) == 3 * sizeof(float), "Color must be 3 packed floats");
    return rt_render(c.handle, &cam, depth, &opts, reinterpret_cast<float*>(buffer.buf.data()), nullptr);
}

// ---------------------------------------------------------------- scenes

// my_scene.rs:11-43: dim_white = 0.1 * WHITE; checkerboard as a texture program.
static Texture dim_white() { return Texture::constant(0.1f * colors::WHITE); }

void create_scene(Scene& scene) {  // my_scene.rs:45-120
    using namespace colors;
    const Color DIM_WHITE(0.1f, 0.1f, 0.1f);
    const Color DIM_BLUE(0.f, 0.f, 0.1f);

    auto phong = Phong(DIM_WHITE, RED, WHITE, 60.f, 0.5f, 0.f);
    Shape sph = Sphere(phong);
    sph.set_transform(Matrix::translate(-1.0f, 0.f, 0.f) * Matrix::rotate_z(75.f) *
                      Matrix::scale(1.0f, 0.25f, 1.0f));
    scene.add_shape(sph);

    phong = Phong(BLACK, BLUE, DIM_BLUE, 600.f, 0.4f, 0.f);
    Shape sph2 = SphereWithName("blue", phong);
    sph2.set_transform(Matrix::translate(1.f, -1.f, 0.f));
    scene.add_shape(sph2);

    phong = Phong(BLACK, WHITE, WHITE, 60.f, 0.7f, 1.333f);
    Shape sph4 = Sphere(phong);
    sph4.set_transform(Matrix::translate(0.f, -0.5f, -3.f) * Matrix::scale(0.6f, 0.6f, 0.6f));
    scene.add_shape(sph4);

    auto plane_material = TexturePhong(dim_white(), Texture::checkerboard(), dim_white(), 60.f, 0.f, 0.f);
    scene.add_shape(Plane(Point3(0.f, -2.f, 2.f), Vector3(0.f, 0.f, -1.f), plane_material));

    plane_material = TexturePhong(dim_white(), Texture::checkerboard(), dim_white(), 60.f, 0.f, 0.f);
    scene.add_shape(Plane(Point3(0.f, -2.f, 0.f), Vector3(0.f, 1.f, 0.f), plane_material));

    auto cube_material = Phong(BLACK, WHITE, WHITE, 60.f, 0.f, 1.333f);
    Shape cube = Cube(cube_material);
    cube.set_transform(Matrix::translate(-1.f, -1.0f, -4.f) * Matrix::rotate_x(-45.0f));
    scene.add_shape(cube);

    scene.add_light(PointLight(Point3(4.f, 4.0f, 0.f), Color(1.f, 0.f, 0.f)));
    scene.add_light(PointLight(Point3(-1.f, 2.0f, -4.f), Color(0.f, 1.f, 0.f)));
    scene.add_light(PointLight(Point3(0.f, 8.0f, -4.f), Color(0.f, 0.f, 1.f)));
    scene.set_ambient(Color(0.1f, 0.1f, 0.1f));
}

void create_bench_128_scene(Scene& scene) {  // render.rs:240-246
    using namespace colors;
    Shape sph = Sphere(Phong(WHITE, RED, WHITE, 60.f, 1.f, 0.f));
    sph.set_transform(Matrix::scale(1.0f, 2.25f, 1.0f));
    scene.add_shape(sph);
}

// splitmix64 (Steele, Lea & Flood 2014); uniform f32 in [0,1) from the top 24 bits.
struct SplitMix64 {
    uint64_t s;
    explicit SplitMix64(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    float unit() { return (float)(next() >> 40) * (1.0f / 16777216.0f); }
    float uniform(float a, float b) { return a + (b - a) * unit(); }
    // draws are sequenced x, y, z (C++ leaves argument evaluation order unspecified)
    Point3 point(float x0, float x1, float y0, float y1, float z0, float z1) {
        Point3 p;
        p.x = uniform(x0, x1);
        p.y = uniform(y0, y1);
        p.z = uniform(z0, z1);
        return p;
    }
    Color color(float a, float b) {
        Color c;
        c.r = uniform(a, b);
        c.g = uniform(a, b);
        c.b = uniform(a, b);
        return c;
    }
};

static MaterialRef synth_material(SplitMix64& rng) {
    using namespace colors;
    float pick = rng.unit();
    Color kd = rng.color(0.2f, 1.f);
    if (pick < 0.5f) return Phong(0.1f * kd, kd, WHITE, 60.f, 0.f, 0.f);       // matte
    if (pick < 0.8f) return Phong(BLACK, kd, WHITE, 60.f, 0.5f, 0.f);           // mirror
    return Phong(BLACK, WHITE, WHITE, 60.f, 0.7f, 1.333f);                      // glass (my_scene.rs:64-66)
}

void create_synth_scene(Scene& scene, const rt_synth_params& p) {
    using namespace colors;
    SplitMix64 rng(p.seed);
    for (uint32_t k = 0; k < p.n_spheres; k++) {
        Point3 c = rng.point(-3.f, 3.f, -1.9f, 2.5f, -3.f, 1.5f);
        float r = rng.uniform(p.r_min, p.r_max);
        bool squashed = rng.unit() < 0.1f;
        float theta = rng.uniform(0.f, 180.f);
        Shape s = Sphere(synth_material(rng));
        if (squashed)
            s.set_transform(Matrix::translate(c.x, c.y, c.z) * Matrix::scale(r, 0.5f * r, r) *
                            Matrix::rotate_z(theta));
        else
            s.set_transform(Matrix::translate(c.x, c.y, c.z) * Matrix::scale(r, r, r));
        scene.add_shape(s);
    }
    for (uint32_t k = 0; k < p.n_cubes; k++) {
        Point3 c = rng.point(-3.f, 3.f, -1.9f, 2.5f, -3.f, 1.5f);
        float ang = rng.uniform(-60.f, 60.f);
        float sc = rng.uniform(0.2f, 0.5f);
        bool glass = rng.unit() < 0.2f;
        MaterialRef m = glass ? Phong(BLACK, WHITE, WHITE, 60.f, 0.f, 1.333f)  // my_scene.rs:102-107
                              : synth_material(rng);
        Shape s = Cube(m);
        s.set_transform(Matrix::translate(c.x, c.y, c.z) * Matrix::rotate_x(ang) * Matrix::scale(sc, sc, sc));
        scene.add_shape(s);
    }
    for (uint32_t k = 0; k < p.n_triangles; k++) {
        Point3 a = rng.point(-3.f, 3.f, -1.9f, 2.5f, -3.f, 1.5f);
        Point3 db = rng.point(-0.3f, 0.3f, -0.3f, 0.3f, -0.3f, 0.3f);
        Point3 dc = rng.point(-0.3f, 0.3f, -0.3f, 0.3f, -0.3f, 0.3f);
        Point3 b(a.x + db.x, a.y + db.y, a.z + db.z);
        Point3 c(a.x + dc.x, a.y + dc.y, a.z + dc.z);
        scene.add_shape(Triangle(a, b, c, synth_material(rng)));
    }
    // my_scene.rs:71-99 planes and :110-118 lights + ambient
    auto pm = TexturePhong(dim_white(), Texture::checkerboard(), dim_white(), 60.f, 0.f, 0.f);
    scene.add_shape(Plane(Point3(0.f, -2.f, 2.f), Vector3(0.f, 0.f, -1.f), pm));
    pm = TexturePhong(dim_white(), Texture::checkerboard(), dim_white(), 60.f, 0.f, 0.f);
    scene.add_shape(Plane(Point3(0.f, -2.f, 0.f), Vector3(0.f, 1.f, 0.f), pm));
    scene.add_light(PointLight(Point3(4.f, 4.0f, 0.f), Color(1.f, 0.f, 0.f)));
    scene.add_light(PointLight(Point3(-1.f, 2.0f, -4.f), Color(0.f, 1.f, 0.f)));
    scene.add_light(PointLight(Point3(0.f, 8.0f, -4.f), Color(0.f, 0.f, 1.f)));
    scene.set_ambient(Color(0.1f, 0.1f, 0.1f));
}

}  // namespace rust_tracer

// ---------------------------------------------------------------- rt_scenes.h exports

using namespace rust_tracer;

namespace {
// A description plus the arrays it points at, handed out as the rt_scene_desc* (first member).
struct OwnedDesc {  // standard layout: `desc` is at offset 0
    rt_scene_desc desc;
    Scene::Flat* flat;
};
rt_status hand_out(const Scene& s, rt_scene_desc** out) {
    if (!out) return RT_ERR_INVALID_ARG;
    OwnedDesc* d = new OwnedDesc();
    d->flat = s.flatten().release();
    d->desc = d->flat->desc;
    *out = &d->desc;
    return RT_OK;
}
}  // namespace

extern "C" {

rt_status rt_desc_my_scene(rt_scene_desc** out) {
    Scene s;
    create_scene(s);
    return hand_out(s, out);
}

rt_status rt_desc_bench_128(rt_scene_desc** out) {
    Scene s;
    create_bench_128_scene(s);
    return hand_out(s, out);
}

rt_status rt_desc_synth(const rt_synth_params* p, rt_scene_desc** out) {
    if (!p) return RT_ERR_INVALID_ARG;
    Scene s;
    create_synth_scene(s, *p);
    return hand_out(s, out);
}

rt_status rt_synth_config(int32_t config, rt_synth_params* out) {
    if (!out) return RT_ERR_INVALID_ARG;
    std::memset(out, 0, sizeof(*out));
    if (config == 2) {
        out->seed = 1; out->n_spheres = 100; out->r_min = 0.15f; out->r_max = 0.45f;
        return RT_OK;
    }
    if (config >= 3 && config <= 5) {
        out->seed = 2; out->n_spheres = 600; out->n_cubes = 25; out->n_triangles = 100;
        out->r_min = 0.06f; out->r_max = 0.2f;
        return RT_OK;
    }
    return RT_ERR_INVALID_ARG;
}

rt_status rt_mirror_render_calls(int32_t scene_id, uint32_t x_res, uint32_t y_res, uint32_t depth, uint32_t n_calls,
                                 int32_t edit, int32_t device, float* ms, int32_t* updates, float* rgb,
                                 float* rgb_fresh) {
    if (n_calls == 0 || x_res == 0 || y_res == 0 || edit < 0 || edit > 3 || (edit && n_calls < 2))
        return RT_ERR_INVALID_ARG;
    Scene scene;
    if (scene_id == 0) {
        create_scene(scene);
    } else {
        rt_synth_params p;
        if (rt_synth_config(scene_id, &p) != RT_OK) return RT_ERR_INVALID_ARG;
        create_synth_scene(scene, p);
    }
    Camera camera(x_res, y_res);
    RenderBuffer buffer(x_res, y_res);
    for (uint32_t k = 0; k < n_calls; k++) {
        if (edit && k + 1 == n_calls) {
            if (edit == 1) {
                Shape* s = scene.find_shape_mut("Sphere");
                if (!s) return RT_ERR_INVALID_ARG;
                s->set_transform(Matrix::translate(0.1f, 0.f, 0.f) * s->transform);
            } else if (edit == 2) {
                // (reflectivity is only a switch in trace_ray, render.rs:70: the diffuse colour
                // changes the lights' and refracted terms)
                scene.shapes().front().material->diffuse = Texture::constant(Color(0.25f, 0.5f, 0.75f));
            } else {
                scene.add_light(PointLight(Point3(-3.f, 5.f, -6.f), Color(0.3f, 0.3f, 0.3f)));
            }
        }
        auto t0 = std::chrono::steady_clock::now();
        int32_t what = 0;
        rt_status st = render(camera, scene, buffer, depth, device, nullptr, nullptr, &what);
        if (st != RT_OK) return st;
        if (ms) ms[k] = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (updates) updates[k] = what;
    }
    const size_t n = (size_t)x_res * y_res * 3;
    if (rgb) std::memcpy(rgb, buffer.buf.data(), n * sizeof(float));
    if (rgb_fresh) {
        Scene copy(scene);  // a Scene of its own: a newly created device handle
        RenderBuffer fresh(x_res, y_res);
        int32_t what = 0;
        rt_status st = render(camera, copy, fresh, depth, device, nullptr, nullptr, &what);
        if (st != RT_OK) return st;
        if (what != -1) return RT_ERR_INVALID_ARG;
        std::memcpy(rgb_fresh, fresh.buf.data(), n * sizeof(float));
    }
    return RT_OK;
}

void rt_desc_free(rt_scene_desc* desc) {
    if (!desc) return;
    OwnedDesc* d = reinterpret_cast<OwnedDesc*>(desc);  // desc is the first member
    delete d->flat;
    delete d;
}

}  // extern "C"
