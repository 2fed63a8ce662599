// rt_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see oracle_api.h).
//
// A CPU restatement of the reference render path, kept in the reference's own
// object model (trait objects -> virtual classes, Rc<RefCell<Material>> ->
// shared_ptr<Material>) so that every floating-point expression is evaluated in
// the order the Rust source writes it.  Compiled with -O2 -ffp-contract=off and
// no fast-math: rustc never contracts a*b+c into an FMA, and glibc libm is the
// libm Rust std links for powf/atan2f/acosf.
//
// One documented choice: Matrix::rotate_{x,y,z} take cos/sin of an f32 angle.  In a
// release build rustc inlines rotate_z(75.) etc. and LLVM constant-folds
// llvm.cos.f32 by evaluating cos() in double and rounding to f32; we evaluate
// (float)cos((double)rads) everywhere to match that (<= 1 ulp vs runtime cosf).
//
// Parity status: pinned by the reference's unit tests (restated in
// tests/test_oracle_kat.py); full frames are "parity unpinned by reference tests"
//  because the reference has no render-output test or golden image.

#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <thread>
#include <vector>
#include <set>
#include <functional>
#include <string>

#include "oracle_api.h"

namespace oracle {

static const float EPS = std::numeric_limits<float>::epsilon();  // std::f32::EPSILON
static const float PI_F = 3.14159265358979323846f;                 // std::f32::consts::PI

// ---------------------------------------------------------------- math (src/math)

struct Vector3 {  // vector3.rs:6-116
    float x, y, z;
    Vector3() : x(0), y(0), z(0) {}
    Vector3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
    Vector3 neg() const { return Vector3(-x, -y, -z); }                           // :30
    Vector3 scalar_mul(float a) const { return Vector3(x * a, y * a, z * a); }    // :39
    Vector3 scalar_div(float d) const { return Vector3(x / d, y / d, z / d); }    // :48
    Vector3 add(const Vector3& v) const { return Vector3(x + v.x, y + v.y, z + v.z); }
    Vector3 sub(const Vector3& v) const { return Vector3(x - v.x, y - v.y, z - v.z); }
    float len2() const { return x * x + y * y + z * z; }                          // :75
    float len() const { return std::sqrt(len2()); }                               // :80
    float dot(const Vector3& v) const { return x * v.x + y * v.y + z * v.z; }     // :86
    Vector3 norm() const { return scalar_div(len()); }                            // :91
    Vector3 cross(const Vector3& v) const {                                       // :97
        return Vector3(y * v.z - z * v.y, z * v.x - x * v.z, x * v.y - y * v.x);
    }
    // vector3.rs:113-115: 2. * (self.dot(about)) * about - self
    Vector3 reflect(const Vector3& about) const {
        float s = 2.f * dot(about);
        return about.scalar_mul(s).sub(*this);
    }
};

struct Point3 {  // point.rs
    float x, y, z;
    Point3() : x(0), y(0), z(0) {}
    Point3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
    Vector3 sub(const Point3& q) const { return Vector3(x - q.x, y - q.y, z - q.z); }  // :38
    Point3 add(const Vector3& v) const { return Point3(x + v.x, y + v.y, z + v.z); }   // :42
    Vector3 as_vec() const { return Vector3(x, y, z); }  // From<Point3> for Vector3
};

struct Ray {  // ray.rs
    Point3 o;
    Vector3 d;
    Ray() {}
    Ray(const Point3& o_, const Vector3& d_) : o(o_), d(d_) {}
    Point3 at(float t) const { return o.add(d.scalar_mul(t)); }  // scalar_mul :50 (`t * ray`)
};

struct Matrix {  // matrix.rs, row-major
    float m[4][4];
    static Matrix zero() { Matrix r; std::memset(r.m, 0, sizeof(r.m)); return r; }
    static Matrix identity() {
        Matrix r = zero();
        for (int i = 0; i < 4; i++) r.m[i][i] = 1.f;
        return r;
    }
    static Matrix from(const float* a) { Matrix r; std::memcpy(r.m, a, sizeof(r.m)); return r; }
    void store(float* a) const { std::memcpy(a, m, sizeof(m)); }
    Matrix mul(const Matrix& a) const {  // mat_mul :68-86 (sum from 0., i = 0..3)
        Matrix r;
        for (int row = 0; row < 4; row++)
            for (int col = 0; col < 4; col++) {
                float s = 0.f;
                for (int i = 0; i < 4; i++) s += m[row][i] * a.m[i][col];
                r.m[row][col] = s;
            }
        return r;
    }
    Matrix transpose() const {
        Matrix r;
        for (int row = 0; row < 4; row++)
            for (int col = 0; col < 4; col++) r.m[row][col] = m[col][row];
        return r;
    }
    // invert :105-153, Gauss-Jordan that pivots only when |diag| < EPS and skips the
    // elimination of a row whose coefficient is below EPS.  Returns false on the
    // reference's panic("Singular Matrix").
    bool invert() {
        Matrix inv = identity();
        for (int col = 0; col < 4; col++) {
            if (std::fabs(m[col][col]) < EPS) {
                int big = col;
                for (int row = 0; row < 4; row++)
                    if (std::fabs(m[row][col]) > std::fabs(m[big][col])) big = row;
                if (big == col) return false;
                for (int j = 0; j < 4; j++) {
                    std::swap(m[big][j], m[col][j]);
                    std::swap(inv.m[big][j], inv.m[col][j]);
                }
            }
            for (int row = 0; row < 4; row++) {
                if (row == col) continue;
                float coeff = m[row][col] / m[col][col];
                if (std::fabs(coeff) >= EPS) {
                    for (int j = 0; j < 4; j++) {
                        m[row][j] -= coeff * m[col][j];
                        inv.m[row][j] -= coeff * inv.m[col][j];
                    }
                    m[row][col] = 0.f;
                }
            }
        }
        for (int row = 0; row < 4; row++)
            for (int col = 0; col < 4; col++) inv.m[row][col] /= m[row][row];
        std::memcpy(m, inv.m, sizeof(m));
        return true;
    }
    static Matrix scale(float x, float y, float z) {
        Matrix r = identity();
        r.m[0][0] = x; r.m[1][1] = y; r.m[2][2] = z;
        return r;
    }
    static Matrix translate(float x, float y, float z) {
        Matrix r = identity();
        r.m[0][3] = x; r.m[1][3] = y; r.m[2][3] = z;
        return r;
    }
    static float rad(float angle) { return angle / 180.0f * PI_F; }
    static float fcos(float r) { return (float)std::cos((double)r); }
    static float fsin(float r) { return (float)std::sin((double)r); }
    static Matrix rotate_x(float a) {  // :177-189
        float r = rad(a);
        Matrix q = identity();
        q.m[1][1] = fcos(r); q.m[1][2] = -fsin(r);
        q.m[2][1] = fsin(r); q.m[2][2] = fcos(r);
        return q;
    }
    static Matrix rotate_y(float a) {  // :191-203
        float r = rad(a);
        Matrix q = identity();
        q.m[0][0] = fcos(r); q.m[0][2] = fsin(r);
        q.m[2][0] = -fsin(r); q.m[2][2] = fcos(r);
        return q;
    }
    static Matrix rotate_z(float a) {  // :205-217
        float r = rad(a);
        Matrix q = identity();
        q.m[0][0] = fcos(r); q.m[0][1] = -fsin(r);
        q.m[1][0] = fsin(r); q.m[1][1] = fcos(r);
        return q;
    }
    Vector3 vec3_mul(const Vector3& v) const {  // :240-246
        return Vector3(v.x * m[0][0] + v.y * m[0][1] + v.z * m[0][2],
                       v.x * m[1][0] + v.y * m[1][1] + v.z * m[1][2],
                       v.x * m[2][0] + v.y * m[2][1] + v.z * m[2][2]);
    }
    Point3 pt_mul(const Point3& p) const {  // :248-263
        return Point3(p.x * m[0][0] + p.y * m[0][1] + p.z * m[0][2] + m[0][3],
                      p.x * m[1][0] + p.y * m[1][1] + p.z * m[1][2] + m[1][3],
                      p.x * m[2][0] + p.y * m[2][1] + p.z * m[2][2] + m[2][3]);
    }
    Ray ray_mul(const Ray& r) const { return Ray(pt_mul(r.o), vec3_mul(r.d)); }  // :265-267
};

// Vector3::mat_mul / Point3::mat_mul (row-vector forms; not on the render path, KATs only)
static Vector3 vec3_mat_mul(const Vector3& v, const Matrix& a) {
    return Vector3(v.x * a.m[0][0] + v.y * a.m[1][0] + v.z * a.m[2][0],
                   v.x * a.m[0][1] + v.y * a.m[1][1] + v.z * a.m[2][1],
                   v.x * a.m[0][2] + v.y * a.m[1][2] + v.z * a.m[2][2]);
}
static Point3 pt_mat_mul(const Point3& p, const Matrix& a) {
    return Point3(p.x * a.m[0][0] + p.y * a.m[1][0] + p.z * a.m[2][0] + a.m[3][0],
                  p.x * a.m[0][1] + p.y * a.m[1][1] + p.z * a.m[2][1] + a.m[3][1],
                  p.x * a.m[0][2] + p.y * a.m[1][2] + p.z * a.m[2][2] + a.m[3][2]);
}

// ---------------------------------------------------------------- colour (color.rs)

struct Color {
    float r, g, b;
    Color() : r(0), g(0), b(0) {}
    Color(float r_, float g_, float b_) : r(r_), g(g_), b(b_) {}
    Color operator+(const Color& o) const { return Color(r + o.r, g + o.g, b + o.b); }
    Color operator*(const Color& o) const { return Color(r * o.r, g * o.g, b * o.b); }
    Color& operator+=(const Color& o) { r += o.r; g += o.g; b += o.b; return *this; }
};
static Color scale(float s, const Color& c) { return Color(s * c.r, s * c.g, s * c.b); }  // f32 * Color
static const Color BLACK(0, 0, 0);
static const Color WHITE(1, 1, 1);

// `as u8` on f32 is saturating in Rust (NaN -> 0)
static uint8_t sat_u8(float x) {
    if (!(x > 0.f)) return 0;  // NaN and negatives
    if (x >= 255.f) return 255;
    return (uint8_t)x;
}
static int32_t sat_i32(float x) {
    if (std::isnan(x)) return 0;
    if (x >= 2147483648.f) return INT32_MAX;
    if (x <= -2147483648.f) return INT32_MIN;
    return (int32_t)x;
}

typedef std::pair<float, float> TexCoords;

// my_scene.rs:26-43
static Color checkerboard(TexCoords tx) {
    int32_t u = sat_i32(std::fabs(tx.first));
    int32_t v = sat_i32(std::fabs(tx.second));
    Color half = scale(0.5f, WHITE);
    if ((tx.first < 0.f && tx.second < 0.f) || (tx.first > 0.f && tx.second > 0.f)) {
        return (u % 2 == v % 2) ? WHITE : half;
    } else {
        return (u % 2 != v % 2) ? WHITE : half;
    }
}

// ---------------------------------------------------------------- materials (material.rs)

struct Intersection;

struct Material {
    virtual ~Material() {}
    virtual Color get_reflected_energy(const Color& incoming, const Vector3& ldir,
                                       const Intersection& i) const = 0;
    virtual Color diffuse(TexCoords tx) const = 0;
    virtual Color ambient(TexCoords tx) const = 0;
    virtual float reflectivity() const = 0;
    virtual float refraction_index() const = 0;
};

struct Intersection {  // intersection.rs:7-17
    int32_t id = 0;
    float t = 0;
    std::shared_ptr<Material> material;
    Point3 point;
    Vector3 eye_dir;
    Vector3 normal;
    bool entering = false;
    TexCoords tex_coord{0.f, 0.f};
};

// material.rs:193-195
static Color lambert(const Vector3& ldir, const Vector3& n, const Color& light, const Color& surface) {
    return scale(ldir.dot(n), light) * surface;
}
// material.rs:197-213
static Color phong(float power, const Vector3& eye, const Vector3& ldir, const Vector3& n,
                   const Color& light, const Color& surface) {
    Vector3 h = eye.norm().add(ldir.norm()).norm();
    float m_dot_h = n.dot(h);
    if (m_dot_h < 0.f) return BLACK;
    return scale(std::pow(m_dot_h, power), light) * surface;
}

struct Phong : Material {  // material.rs:24-101
    Color ka, kd, ks;
    float power, refl, ri;
    Phong(Color a, Color d, Color s, float p, float r, float i)
        : ka(a), kd(d), ks(s), power(p), refl(r), ri(i) {}
    Color diffuse(TexCoords) const override { return kd; }
    Color ambient(TexCoords) const override { return ka; }
    float reflectivity() const override { return refl; }
    float refraction_index() const override { return ri; }
    Color get_reflected_energy(const Color& e, const Vector3& l, const Intersection& i) const override {
        Color d = lambert(l, i.normal, e, kd);
        Color s = phong(power, i.eye_dir, l, i.normal, e, ks);
        return d + s;
    }
};

typedef std::function<Color(TexCoords)> ColorFun;

struct TexturePhong : Material {  // material.rs:103-191
    ColorFun fa, fd, fs;
    float power, refl, ri;
    TexturePhong(ColorFun a, ColorFun d, ColorFun s, float p, float r, float i)
        : fa(a), fd(d), fs(s), power(p), refl(r), ri(i) {}
    Color diffuse(TexCoords tx) const override { return fd(tx); }
    Color ambient(TexCoords tx) const override { return fa(tx); }
    float reflectivity() const override { return refl; }
    float refraction_index() const override { return ri; }
    Color get_reflected_energy(const Color& e, const Vector3& l, const Intersection& i) const override {
        Color d = lambert(l, i.normal, e, fd(i.tex_coord));
        Color s = phong(power, i.eye_dir, l, i.normal, e, fs(i.tex_coord));
        return d + s;
    }
};

// ---------------------------------------------------------------- shapes (scene/*.rs)

struct Renderable {
    int32_t id = 0;
    virtual ~Renderable() {}
    virtual bool intersect(const Ray& ray, Intersection& out) const = 0;
    virtual bool set_transform(const Matrix& m) = 0;
    virtual size_t size() const { return 1; }
    std::string name;
};

// sphere.rs:126-145
static bool solve_quadratic(float a, float b, float c, float& x0, float& x1) {
    float discr = b * b - 4.f * a * c;
    if (discr < 0.f) return false;
    if (std::fabs(discr) < EPS) {
        float x = -0.5f * b / a;
        x0 = x; x1 = x;
        return true;
    }
    float q = (b > 0.f) ? -0.5f * (b + std::sqrt(discr)) : -0.5f * (b - std::sqrt(discr));
    x0 = q / a;
    x1 = c / q;
    return true;
}

struct Sphere : Renderable {  // sphere.rs
    Matrix transform = Matrix::identity(), inv = Matrix::identity();
    std::shared_ptr<Material> material;
    explicit Sphere(std::shared_ptr<Material> m) : material(m) { name = "Sphere"; }
    static TexCoords tex(const Vector3& n) {  // :40-45
        float u = (1.f + std::atan2(n.z, n.x) / PI_F) * 0.5f;
        float v = std::acos(n.y) / PI_F;
        return TexCoords(u, v);
    }
    bool intersect(const Ray& ray, Intersection& out) const override {  // :57-98
        Ray tr = inv.ray_mul(ray);
        Vector3 l = tr.o.sub(Point3(0.f, 0.f, 0.f));
        float a = tr.d.len2();
        float b = 2.f * tr.d.dot(l);
        float c = l.len2() - 1.f;
        float t0, t1;
        if (!solve_quadratic(a, b, c, t0, t1)) return false;
        if (t0 > t1) std::swap(t0, t1);
        if (t0 < 0.f && t1 < 0.f) return false;
        float t = (t0 < 0.f) ? t1 : t0;
        bool entering = t0 > 0.f;
        Point3 point = ray.at(t);
        Point3 onrm = tr.at(t);
        Vector3 normal = inv.transpose().vec3_mul(onrm.as_vec()).norm();
        if (!entering) normal = normal.neg();
        out.id = id;
        out.t = t;
        out.material = material;
        out.point = point;
        out.eye_dir = ray.d.norm().neg();
        out.normal = normal;
        out.entering = entering;
        out.tex_coord = tex(normal);
        return true;
    }
    bool set_transform(const Matrix& m) override {
        transform = m;
        inv = m;
        return inv.invert();
    }
};

struct Triangle : Renderable {  // triangle.rs
    Point3 v[3];
    Vector3 normal;
    Matrix transform = Matrix::identity(), inv = Matrix::identity();
    std::shared_ptr<Material> material;
    Triangle(const Point3& a, const Point3& b, const Point3& c, std::shared_ptr<Material> m)
        : material(m) {
        v[0] = a; v[1] = b; v[2] = c;
        Vector3 v0v1 = b.sub(a);
        Vector3 v0v2 = c.sub(b);  // sic: v2 - v1 (triangle.rs:27)
        normal = v0v1.cross(v0v2).norm();
        name = "Triable";
    }
    bool intersect(const Ray& ray, Intersection& out) const override {  // :51-94
        Vector3 v0v1 = v[1].sub(v[0]);
        Vector3 v0v2 = v[2].sub(v[0]);
        Vector3 pvec = ray.d.cross(v0v2);
        float det = v0v1.dot(pvec);
        if (std::fabs(det) < EPS) return false;
        float inv_det = 1.0f / det;
        Vector3 tvec = ray.o.sub(v[0]);
        float u = tvec.dot(pvec) * inv_det;
        if (u < 0.f || u > 1.f) return false;
        Vector3 qvec = tvec.cross(v0v1);
        float vv = ray.d.dot(qvec) * inv_det;
        if (vv < 0.f || u + vv > 1.f) return false;
        float t = v0v2.dot(qvec) * inv_det;
        if (t < 0.f) return false;
        out.id = id;
        out.t = t;
        out.material = material;
        out.point = ray.at(t);
        out.eye_dir = ray.d.norm().neg();
        out.normal = normal;  // the t<0 flip at :82 is unreachable
        out.entering = det > 0.f;
        out.tex_coord = TexCoords(u, vv);
        return true;
    }
    bool set_transform(const Matrix& m) override {  // stored, never used by intersect
        transform = m;
        inv = m;
        return inv.invert();
    }
};

struct Scene;

struct Plane : Renderable {  // plane.rs
    Point3 origin;
    Vector3 normal, u, v;
    Matrix transform = Matrix::identity(), inv = Matrix::identity();
    std::shared_ptr<Material> material;
    Plane(const Point3& o, const Vector3& n, std::shared_ptr<Material> m)
        : origin(o), normal(n), material(m) {  // :22-42
        Vector3 w = (n.cross(Vector3(1.f, 0.f, 0.f)).len() <= EPS) ? Vector3(0.f, 1.f, 0.f)
                                                                     : Vector3(1.f, 0.f, 0.f);
        u = n.cross(w).norm();
        v = n.cross(u).norm();
        name = "Plane";
    }
    bool intersect(const Ray& ray, Intersection& out) const override {  // :59-84
        Ray tr = inv.ray_mul(ray);
        float denom = -normal.dot(tr.d);
        if (!(denom > EPS)) return false;
        Vector3 dir = origin.sub(tr.o);
        float t = -dir.dot(normal) / denom;
        Point3 point = ray.at(t);
        out.id = id;
        out.t = t;
        out.entering = t >= 0.f;
        out.point = point;
        out.eye_dir = ray.d.norm().neg();
        out.normal = transform.vec3_mul(normal);
        out.material = material;
        out.tex_coord = TexCoords(u.dot(point.as_vec()), v.dot(point.as_vec()));
        return true;
    }
    bool set_transform(const Matrix& m) override {
        transform = m;
        inv = m;
        return inv.invert();
    }
};

struct LightSource {
    virtual ~LightSource() {}
    virtual std::pair<Vector3, Color> get_energy(const Scene& s, const Point3& p) const = 0;
};

struct Counters {
    uint64_t node_rays = 0, shadow_rays = 0, pixels = 0;
};

struct Scene : Renderable {  // scene/mod.rs:22-137
    Color ambient;
    std::vector<std::unique_ptr<LightSource>> lights;
    std::vector<std::unique_ptr<Renderable>> shapes;
    void add_shape(std::unique_ptr<Renderable> s) {
        s->id = (int32_t)shapes.size();
        shapes.push_back(std::move(s));
    }
    bool set_transform(const Matrix&) override { return true; }
    bool intersect(const Ray& ray, Intersection& out) const override {  // :98-116
        bool found = false;
        float nearest = 0.f;
        Intersection cand;
        for (const auto& s : shapes) {
            if (!s->intersect(ray, cand)) continue;
            if (!found) {
                nearest = cand.t;
                out = cand;
                found = true;
            } else if (cand.t < nearest) {
                nearest = cand.t;
                out = cand;
            }
        }
        return found;
    }
    size_t size() const override {
        size_t n = 0;
        for (const auto& s : shapes) n += s->size();
        return n;
    }
};

struct Cube : Renderable {  // cube.rs
    Scene tris;
    Matrix transform = Matrix::identity(), inv = Matrix::identity();
    explicit Cube(std::shared_ptr<Material> m) {  // :21-77
        Point3 v0(0.5f, 0.5f, -0.5f), v1(0.5f, -0.5f, -0.5f), v2(-0.5f, -0.5f, -0.5f),
            v3(-0.5f, 0.5f, -0.5f), v4(0.5f, 0.5f, 0.5f), v5(-0.5f, 0.5f, 0.5f),
            v6(-0.5f, -0.5f, 0.5f), v7(0.5f, -0.5f, 0.5f);
        auto T = [&](const Point3& a, const Point3& b, const Point3& c) {
            tris.add_shape(std::unique_ptr<Renderable>(new Triangle(a, b, c, m)));
        };
        T(v1, v2, v3); T(v0, v1, v3);  // front  tf1 tf2
        T(v7, v5, v4); T(v5, v7, v6);  // back   tk1 tk2
        T(v0, v4, v7); T(v7, v1, v0);  // right  tr1 tr2
        T(v5, v3, v6); T(v6, v3, v2);  // left   tl1 tl2
        T(v5, v4, v0); T(v0, v3, v5);  // top    tt1 tt2  (added before bottom, :58-69)
        T(v1, v7, v6); T(v6, v2, v1);  // bottom tb1 tb2
        name = "Cube";
    }
    bool intersect(const Ray& ray, Intersection& out) const override {  // :89-102
        Ray tr = inv.ray_mul(ray);
        if (!tris.intersect(tr, out)) return false;
        out.point = ray.at(out.t);
        out.eye_dir = ray.d.norm().neg();
        out.normal = inv.transpose().vec3_mul(out.normal).norm();
        return true;
    }
    bool set_transform(const Matrix& m) override {
        transform = m;
        inv = m;
        return inv.invert();
    }
    size_t size() const override { return tris.size(); }
};

struct PointLight : LightSource {  // mod.rs:178-206
    Point3 pos;
    Color color;
    mutable Counters* counters = nullptr;
    PointLight(Point3 p, Color c) : pos(p), color(c) {}
    std::pair<Vector3, Color> get_energy(const Scene& s, const Point3& point) const override {
        Vector3 dir = pos.sub(point).norm();
        Ray ray(point, dir);
        Intersection i;
        Color e;
        if (s.intersect(ray, i)) {
            e = (i.point.sub(point).len2() < pos.sub(point).len2()) ? BLACK : color;
        } else {
            e = color;
        }
        return std::make_pair(dir, e);
    }
};

struct AmbientLight : LightSource {  // mod.rs:224-246
    Color color;
    explicit AmbientLight(Color c) : color(c) {}
    std::pair<Vector3, Color> get_energy(const Scene&, const Point3&) const override {
        return std::make_pair(Vector3(0.f, 0.f, 0.f), color);
    }
};

// ---------------------------------------------------------------- render.rs

struct Camera {  // render.rs:155-186
    Point3 origin;
    float x_min, x_max, y_min, y_max;
    uint32_t x_res, y_res;
    Ray get_ray(uint32_t u, uint32_t v) const {
        float x_delta = (x_max - x_min) / (float)x_res;
        float y_delta = (y_max - y_min) / (float)y_res;
        float x = x_min + (float)u * x_delta;
        float y = y_max - (float)v * y_delta;
        Point3 vp(x, y, 0.f);
        return Ray(origin, vp.sub(origin).norm());
    }
};

// render.rs:129-134
static float fresnel_reflection(const Vector3& l, const Vector3& n, float n1, float n2) {
    float m_dot_r = l.dot(n);
    float q = (n1 - n2) / (n1 + n2);
    float r0 = q * q;
    float x = 1.f - m_dot_r;
    float x2 = x * x;
    float p5 = x * (x2 * x2);  // powi(5): LLVM's square-and-multiply expansion
    return r0 + (1.f - r0) * p5;
}
static float fresnel_refraction(const Vector3& l, const Vector3& n, float n1, float n2) {
    return 1.f - fresnel_reflection(l, n, n1, n2);
}
// render.rs:105-110
static Ray reflect_ray(const Ray& ray, const Intersection& i) {
    Vector3 rd = ray.d.reflect(i.normal).norm().neg();
    Point3 p = i.point.add(rd.scalar_mul(0.0002f));
    return Ray(p, rd);
}
// render.rs:112-125
static bool refract_ray(const Ray& ray, const Intersection& i, float n1, float n2, Ray& out) {
    float ratio = n1 / n2;
    float m_dot_r = -ray.d.dot(i.normal);
    float cos2 = 1.f - ratio * ratio * (1.f - m_dot_r * m_dot_r);
    if (!(cos2 > 0.f)) return false;
    float c = std::sqrt(cos2);
    Vector3 dir = ray.d.scalar_mul(ratio).add(i.normal.scalar_mul(ratio * m_dot_r - c));
    Point3 p = i.point.add(dir.scalar_mul(0.0002f));
    out = Ray(p, dir);
    return true;
}
// render.rs:142-153 (+ shadow-ray counting)
static std::vector<std::pair<Vector3, Color>> get_light_energy(const Scene& s, const Intersection& i,
                                                               Counters& cnt) {
    Point3 p = i.point.add(i.normal.scalar_mul(0.0002f));
    std::vector<std::pair<Vector3, Color>> out;
    for (const auto& l : s.lights) {
        if (dynamic_cast<const PointLight*>(l.get())) cnt.shadow_rays++;
        out.push_back(l->get_energy(s, p));
    }
    return out;
}

// render.rs:40-103
static Color trace_ray(const Scene& s, const Ray& ray, uint32_t depth, Counters& cnt) {
    if (depth == 0) return BLACK;
    Intersection i;
    cnt.node_rays++;
    if (!s.intersect(ray, i)) return BLACK;
    const Material& m = *i.material;
    float n1 = i.entering ? 1.f : m.refraction_index();
    float n2 = i.entering ? m.refraction_index() : 1.f;
    Color ambient = m.ambient(i.tex_coord) * s.ambient;
    Color lights = BLACK;  // Sum starts at BLACK, color.rs:164-167
    for (const auto& le : get_light_energy(s, i, cnt)) {
        float f = fresnel_reflection(le.first, i.normal, n1, n2);
        lights += scale(f, m.get_reflected_energy(le.second, le.first, i));
    }
    Color reflected = BLACK;
    if (m.reflectivity() > EPS) {
        Ray rr = reflect_ray(ray, i);
        Color e = trace_ray(s, rr, depth - 1, cnt);
        float f = fresnel_reflection(rr.d, i.normal, n1, n2);
        reflected = scale(f, m.get_reflected_energy(e, rr.d, i));
    }
    Color refracted = BLACK;
    if (m.refraction_index() > EPS) {
        Ray tr;
        Color inner = BLACK;
        if (refract_ray(ray, i, n1, n2, tr)) {
            float f = fresnel_refraction(tr.d, i.normal.neg(), n1, n2);
            inner = scale(f, trace_ray(s, tr, depth - 1, cnt));
        }
        refracted = m.diffuse(i.tex_coord) * inner;
    }
    return ambient + lights + reflected + refracted;
}

// ---------------------------------------------------------------- render_tree.rs

struct RayTreeNode {
    Intersection i;
    std::vector<std::pair<Vector3, Color>> lights;
    std::unique_ptr<RayTreeNode> reflected, refracted;
};

// render_tree.rs:166-212
static std::unique_ptr<RayTreeNode> build_ray_tree(const Scene& s, const Ray& ray, uint32_t depth,
                                                   std::set<int32_t>& shapes, Counters& cnt) {
    if (depth == 0) return nullptr;
    Intersection i;
    cnt.node_rays++;
    if (!s.intersect(ray, i)) return nullptr;
    shapes.insert(i.id);
    const Material& m = *i.material;
    float n1 = i.entering ? 1.f : m.refraction_index();
    float n2 = i.entering ? m.refraction_index() : 1.f;
    std::unique_ptr<RayTreeNode> node(new RayTreeNode());
    node->lights = get_light_energy(s, i, cnt);
    if (m.reflectivity() > EPS) node->reflected = build_ray_tree(s, reflect_ray(ray, i), depth - 1, shapes, cnt);
    if (m.refraction_index() > EPS) {
        Ray tr;
        if (refract_ray(ray, i, n1, n2, tr)) node->refracted = build_ray_tree(s, tr, depth - 1, shapes, cnt);
    }
    node->i = i;
    return node;
}

// render_tree.rs:214-255
static std::pair<Color, Vector3> render_ray_tree(const RayTreeNode* node, const Color& amb) {
    if (!node) return std::make_pair(BLACK, Vector3(0.f, 0.f, 0.f));
    const Intersection& i = node->i;
    const Material& m = *i.material;
    float n1 = i.entering ? 1.f : m.refraction_index();
    float n2 = i.entering ? m.refraction_index() : 1.f;
    Color lights = BLACK;
    for (const auto& le : node->lights) {
        float f = fresnel_reflection(le.first, i.normal, n1, n2);
        lights += scale(f, m.get_reflected_energy(le.second, le.first, i));
    }
    auto rl = render_ray_tree(node->reflected.get(), amb);
    float fr = fresnel_reflection(rl.second, i.normal, n1, n2);
    Color reflected = scale(fr, m.get_reflected_energy(rl.first, i.eye_dir, i));
    auto rf = render_ray_tree(node->refracted.get(), amb);
    float ft = fresnel_refraction(rf.second, i.normal.neg(), n1, n2);
    Color refracted = scale(ft, rf.first);
    Color ambient = m.ambient(i.tex_coord) * amb;
    return std::make_pair(ambient + lights + reflected + refracted, i.eye_dir.neg());
}

static uint32_t tree_size(const RayTreeNode* n) {  // render_tree.rs:39-48
    return n ? 1 + tree_size(n->reflected.get()) + tree_size(n->refracted.get()) : 0;
}

// ---------------------------------------------------------------- my_scene.rs:45-120

static Color dim_white(TexCoords) { return scale(0.1f, WHITE); }

static bool create_my_scene(Scene& scene) {
    const Color DIM_WHITE(0.1f, 0.1f, 0.1f), DIM_BLUE(0.f, 0.f, 0.1f);
    const Color RED(1.f, 0.f, 0.f), BLUE(0.f, 0.f, 1.f);
    bool ok = true;
    {
        auto m = std::make_shared<Phong>(DIM_WHITE, RED, WHITE, 60.f, 0.5f, 0.f);
        auto s = std::unique_ptr<Sphere>(new Sphere(m));
        ok &= s->set_transform(Matrix::translate(-1.0f, 0.f, 0.f).mul(Matrix::rotate_z(75.f))
                                   .mul(Matrix::scale(1.0f, 0.25f, 1.0f)));
        scene.add_shape(std::move(s));
    }
    {
        auto m = std::make_shared<Phong>(BLACK, BLUE, DIM_BLUE, 600.f, 0.4f, 0.f);
        auto s = std::unique_ptr<Sphere>(new Sphere(m));
        s->name = "blue";
        ok &= s->set_transform(Matrix::translate(1.f, -1.f, 0.f));
        scene.add_shape(std::move(s));
    }
    {
        auto m = std::make_shared<Phong>(BLACK, WHITE, WHITE, 60.f, 0.7f, 1.333f);
        auto s = std::unique_ptr<Sphere>(new Sphere(m));
        ok &= s->set_transform(Matrix::translate(0.f, -0.5f, -3.f).mul(Matrix::scale(0.6f, 0.6f, 0.6f)));
        scene.add_shape(std::move(s));
    }
    {
        auto m = std::make_shared<TexturePhong>(dim_white, checkerboard, dim_white, 60.f, 0.f, 0.f);
        scene.add_shape(std::unique_ptr<Renderable>(
            new Plane(Point3(0.f, -2.f, 2.f), Vector3(0.f, 0.f, -1.f), m)));
    }
    {
        auto m = std::make_shared<TexturePhong>(dim_white, checkerboard, dim_white, 60.f, 0.f, 0.f);
        scene.add_shape(std::unique_ptr<Renderable>(
            new Plane(Point3(0.f, -2.f, 0.f), Vector3(0.f, 1.f, 0.f), m)));
    }
    {
        auto m = std::make_shared<Phong>(BLACK, WHITE, WHITE, 60.f, 0.f, 1.333f);
        auto c = std::unique_ptr<Cube>(new Cube(m));
        ok &= c->set_transform(Matrix::translate(-1.f, -1.0f, -4.f).mul(Matrix::rotate_x(-45.0f)));
        scene.add_shape(std::move(c));
    }
    scene.lights.emplace_back(new PointLight(Point3(4.f, 4.0f, 0.f), Color(1.f, 0.f, 0.f)));
    scene.lights.emplace_back(new PointLight(Point3(-1.f, 2.0f, -4.f), Color(0.f, 1.f, 0.f)));
    scene.lights.emplace_back(new PointLight(Point3(0.f, 8.0f, -4.f), Color(0.f, 0.f, 1.f)));
    scene.ambient = Color(0.1f, 0.1f, 0.1f);
    return ok;
}

// ---------------------------------------------------------------- rt_scene_desc -> Scene

static Color cc(const rt_color& c) { return Color(c.r, c.g, c.b); }

static ColorFun texfun(const rt_texture& t) {
    if (t.kind == RT_TEX_CHECKERBOARD) return checkerboard;
    Color c = cc(t.color);
    return [c](TexCoords) { return c; };
}

static rt_status from_desc(const rt_scene_desc* d, Scene& scene, std::vector<std::shared_ptr<Material>>& mats) {
    if (!d) return RT_ERR_INVALID_ARG;
    mats.clear();
    for (uint32_t k = 0; k < d->n_materials; k++) {
        const rt_material& m = d->materials[k];
        if (m.kind == RT_MAT_PHONG) {
            mats.push_back(std::make_shared<Phong>(cc(m.ambient.color), cc(m.diffuse.color),
                                                   cc(m.specular.color), m.power, m.reflectivity,
                                                   m.refraction_index));
        } else if (m.kind == RT_MAT_TEXTURE_PHONG) {
            mats.push_back(std::make_shared<TexturePhong>(texfun(m.ambient), texfun(m.diffuse),
                                                          texfun(m.specular), m.power,
                                                          m.reflectivity, m.refraction_index));
        } else {
            return RT_ERR_INVALID_ARG;
        }
    }
    for (uint32_t k = 0; k < d->n_shapes; k++) {
        const rt_shape& s = d->shapes[k];
        if (s.material < 0 || (uint32_t)s.material >= d->n_materials) return RT_ERR_BAD_MATERIAL;
        auto m = mats[s.material];
        Matrix tf = Matrix::from(s.transform);
        std::unique_ptr<Renderable> r;
        switch (s.kind) {
            case RT_SHAPE_SPHERE: r.reset(new Sphere(m)); break;
            case RT_SHAPE_PLANE:
                r.reset(new Plane(Point3(s.data[0], s.data[1], s.data[2]),
                                  Vector3(s.data[3], s.data[4], s.data[5]), m));
                break;
            case RT_SHAPE_TRIANGLE:
                r.reset(new Triangle(Point3(s.data[0], s.data[1], s.data[2]),
                                     Point3(s.data[3], s.data[4], s.data[5]),
                                     Point3(s.data[6], s.data[7], s.data[8]), m));
                break;
            case RT_SHAPE_CUBE: r.reset(new Cube(m)); break;
            default: return RT_ERR_INVALID_ARG;
        }
        if (!r->set_transform(tf)) return RT_ERR_SINGULAR_MATRIX;
        scene.add_shape(std::move(r));
    }
    for (uint32_t k = 0; k < d->n_lights; k++) {
        const rt_light& l = d->lights[k];
        if (l.kind == RT_LIGHT_POINT)
            scene.lights.emplace_back(new PointLight(Point3(l.pos[0], l.pos[1], l.pos[2]), cc(l.color)));
        else if (l.kind == RT_LIGHT_AMBIENT)
            scene.lights.emplace_back(new AmbientLight(cc(l.color)));
        else
            return RT_ERR_INVALID_ARG;
    }
    scene.ambient = cc(d->ambient);
    return RT_OK;
}

static Camera cam_of(const rt_camera* c) {
    Camera k;
    k.origin = Point3(c->origin[0], c->origin[1], c->origin[2]);
    k.x_min = c->x_min; k.x_max = c->x_max; k.y_min = c->y_min; k.y_max = c->y_max;
    k.x_res = c->x_res; k.y_res = c->y_res;
    return k;
}

static void fill_hit(const Intersection& i, bool hit, oracle_hit* o) {
    std::memset(o, 0, sizeof(*o));
    o->hit = hit ? 1 : 0;
    if (!hit) return;
    o->id = i.id; o->t = i.t;
    o->point[0] = i.point.x; o->point[1] = i.point.y; o->point[2] = i.point.z;
    o->eye_dir[0] = i.eye_dir.x; o->eye_dir[1] = i.eye_dir.y; o->eye_dir[2] = i.eye_dir.z;
    o->normal[0] = i.normal.x; o->normal[1] = i.normal.y; o->normal[2] = i.normal.z;
    o->entering = i.entering ? 1 : 0;
    o->tex[0] = i.tex_coord.first; o->tex[1] = i.tex_coord.second;
}

}  // namespace oracle

using namespace oracle;

struct oracle_scene {
    Scene scene;
    std::vector<std::shared_ptr<Material>> mats;  // by description index (shared with the shapes)
};

// render_tree.rs:51-105: one RayTree per pixel (row-major here), its shape-id set
struct oracle_forest {
    const oracle_scene* s = nullptr;
    uint32_t w = 0, h = 0;
    std::vector<std::unique_ptr<RayTreeNode>> roots;
    std::vector<std::set<int32_t>> shapes;
};

extern "C" {

rt_status oracle_scene_from_desc(const rt_scene_desc* desc, oracle_scene** out) {
    if (!out) return RT_ERR_INVALID_ARG;
    std::unique_ptr<oracle_scene> s(new oracle_scene());
    rt_status st = from_desc(desc, s->scene, s->mats);
    if (st != RT_OK) return st;
    *out = s.release();
    return RT_OK;
}

rt_status oracle_scene_my_scene(oracle_scene** out) {
    if (!out) return RT_ERR_INVALID_ARG;
    std::unique_ptr<oracle_scene> s(new oracle_scene());
    if (!create_my_scene(s->scene)) return RT_ERR_SINGULAR_MATRIX;
    *out = s.release();
    return RT_OK;
}

void oracle_scene_destroy(oracle_scene* s) { delete s; }

rt_status oracle_render_rows(const oracle_scene* s, const rt_camera* cam, uint32_t depth,
                             uint32_t row_begin, uint32_t row_end, uint32_t row_step,
                             float* rgb, uint64_t* counters) {
    if (!s || !cam || !rgb || row_step == 0) return RT_ERR_INVALID_ARG;
    Camera c = cam_of(cam);
    Counters cnt;
    if (row_end > c.y_res) row_end = c.y_res;
    for (uint32_t v = row_begin; v < row_end; v += row_step) {  // render.rs:32-37
        for (uint32_t u = 0; u < c.x_res; u++) {
            Color col = trace_ray(s->scene, c.get_ray(u, v), depth, cnt);
            float* px = rgb + ((size_t)v * c.x_res + u) * 3;
            px[0] = col.r; px[1] = col.g; px[2] = col.b;
            cnt.pixels++;
        }
    }
    if (counters) {
        counters[0] += cnt.node_rays;
        counters[1] += cnt.shadow_rays;
        counters[2] += cnt.pixels;
    }
    return RT_OK;
}

// Stochastic supersampling (no reference equivalent): sample k of
// pixel (u, v) is Camera::get_ray's ray through (u + jx, v + jy), with the counter hash
// of include/rt_api.h (rt_render_spp) restated here; the pixel is the f32 sum of its
// samples in sample order, divided by spp.  spp == 1 is render.rs exactly (no jitter).
static uint32_t spp_mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
static float spp_jitter(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t dim) {
    uint32_t h = spp_mix32(spp_mix32(seed ^ 0x9e3779b9u) ^ pixel);
    h = spp_mix32(h ^ spp_mix32(2u * sample + dim + 1u));
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

rt_status oracle_render_rows_spp(const oracle_scene* s, const rt_camera* cam, uint32_t depth,
                                 uint32_t row_begin, uint32_t row_end, uint32_t row_step,
                                 uint32_t spp, uint32_t seed, float* rgb, uint64_t* counters) {
    if (!s || !cam || !rgb || row_step == 0 || spp == 0) return RT_ERR_INVALID_ARG;
    if (spp == 1) return oracle_render_rows(s, cam, depth, row_begin, row_end, row_step, rgb, counters);
    Camera c = cam_of(cam);
    Counters cnt;
    if (row_end > c.y_res) row_end = c.y_res;
    const float x_delta = (c.x_max - c.x_min) / (float)c.x_res;
    const float y_delta = (c.y_max - c.y_min) / (float)c.y_res;
    for (uint32_t v = row_begin; v < row_end; v += row_step) {
        for (uint32_t u = 0; u < c.x_res; u++) {
            const uint32_t pixel = v * c.x_res + u;
            Color sum(0.f, 0.f, 0.f);
            for (uint32_t k = 0; k < spp; k++) {
                float x = c.x_min + ((float)u + spp_jitter(seed, pixel, k, 0)) * x_delta;
                float y = c.y_max - ((float)v + spp_jitter(seed, pixel, k, 1)) * y_delta;
                Point3 vp(x, y, 0.f);
                Color col = trace_ray(s->scene, Ray(c.origin, vp.sub(c.origin).norm()), depth, cnt);
                if (k == 0) {
                    sum = col;
                } else {
                    sum.r = sum.r + col.r;
                    sum.g = sum.g + col.g;
                    sum.b = sum.b + col.b;
                }
                cnt.pixels++;
            }
            float* px = rgb + ((size_t)v * c.x_res + u) * 3;
            px[0] = sum.r / (float)spp;
            px[1] = sum.g / (float)spp;
            px[2] = sum.b / (float)spp;
        }
    }
    if (counters) {
        counters[0] += cnt.node_rays;
        counters[1] += cnt.shadow_rays;
        counters[2] += cnt.pixels;
    }
    return RT_OK;
}

rt_status oracle_render_rows_mt(const oracle_scene* s, const rt_camera* cam, uint32_t depth,
                                uint32_t row_begin, uint32_t row_end, uint32_t row_step,
                                float* rgb, uint64_t* counters, uint32_t threads) {
    return oracle_render_rows_spp_mt(s, cam, depth, row_begin, row_end, row_step, 1, 0, rgb, counters, threads);
}

rt_status oracle_render_rows_spp_mt(const oracle_scene* s, const rt_camera* cam, uint32_t depth,
                                    uint32_t row_begin, uint32_t row_end, uint32_t row_step, uint32_t spp,
                                    uint32_t seed, float* rgb, uint64_t* counters, uint32_t threads) {
    if (threads <= 1)
        return oracle_render_rows_spp(s, cam, depth, row_begin, row_end, row_step, spp, seed, rgb, counters);
    std::vector<std::thread> pool;
    std::vector<uint64_t> part(3 * threads, 0);
    for (uint32_t k = 0; k < threads; k++) {
        pool.emplace_back([=, &part]() {
            oracle_render_rows_spp(s, cam, depth, row_begin + k * row_step, row_end, row_step * threads,
                                   spp, seed, rgb, &part[3 * k]);
        });
    }
    for (auto& t : pool) t.join();
    if (counters)
        for (uint32_t k = 0; k < threads; k++)
            for (int j = 0; j < 3; j++) counters[j] += part[3 * k + j];
    return RT_OK;
}

rt_status oracle_render_forest(const oracle_scene* s, const rt_camera* cam, uint32_t depth,
                               float* rgb, uint32_t* tree_sizes) {
    if (!s || !cam || !rgb) return RT_ERR_INVALID_ARG;
    Camera c = cam_of(cam);
    Counters cnt;
    for (uint32_t v = 0; v < c.y_res; v++) {
        for (uint32_t u = 0; u < c.x_res; u++) {
            std::set<int32_t> shapes;
            auto tree = build_ray_tree(s->scene, c.get_ray(u, v), depth, shapes, cnt);
            Color col = render_ray_tree(tree.get(), s->scene.ambient).first;
            float* px = rgb + ((size_t)v * c.x_res + u) * 3;
            px[0] = col.r; px[1] = col.g; px[2] = col.b;
            if (tree_sizes) tree_sizes[(size_t)v * c.x_res + u] = tree_size(tree.get());
        }
    }
    return RT_OK;
}

// ---- persistent forest: generate_ray_forest (render_tree.rs:147-164) once, then
// render_forest (:121-127) / render_forest_filter (:129-145) any number of times; the
// trees hold the scene's materials, so oracle_scene_set_material edits show up on the
// next shade exactly as the GUI's RefCell mutations do (gui.rs:221-236)
rt_status oracle_forest_build(const oracle_scene* s, const rt_camera* cam, uint32_t depth, oracle_forest** out) {
    if (!s || !cam || !out) return RT_ERR_INVALID_ARG;
    std::unique_ptr<oracle_forest> f(new oracle_forest());
    Camera c = cam_of(cam);
    f->s = s;
    f->w = c.x_res;
    f->h = c.y_res;
    f->roots.resize((size_t)c.x_res * c.y_res);
    f->shapes.resize((size_t)c.x_res * c.y_res);
    Counters cnt;
    for (uint32_t v = 0; v < c.y_res; v++)
        for (uint32_t u = 0; u < c.x_res; u++) {
            size_t k = (size_t)v * c.x_res + u;
            f->roots[k] = build_ray_tree(s->scene, c.get_ray(u, v), depth, f->shapes[k], cnt);
        }
    *out = f.release();
    return RT_OK;
}

// the same forest built over `threads` host threads (rows dealt in turn; the trees and their
// shape sets are per pixel, the scene is read only -- the Rc<Material> copies are shared_ptr
// copies, whose counts are atomic): test infrastructure for benchmark-size forests
rt_status oracle_forest_build_mt(const oracle_scene* s, const rt_camera* cam, uint32_t depth, uint32_t threads,
                                 oracle_forest** out) {
    if (threads <= 1) return oracle_forest_build(s, cam, depth, out);
    if (!s || !cam || !out) return RT_ERR_INVALID_ARG;
    std::unique_ptr<oracle_forest> f(new oracle_forest());
    Camera c = cam_of(cam);
    f->s = s;
    f->w = c.x_res;
    f->h = c.y_res;
    f->roots.resize((size_t)c.x_res * c.y_res);
    f->shapes.resize((size_t)c.x_res * c.y_res);
    std::vector<std::thread> pool;
    oracle_forest* fp = f.get();
    for (uint32_t k = 0; k < threads; k++)
        pool.emplace_back([=]() {
            Counters cnt;
            for (uint32_t v = k; v < c.y_res; v += threads)
                for (uint32_t u = 0; u < c.x_res; u++) {
                    size_t i = (size_t)v * c.x_res + u;
                    fp->roots[i] = build_ray_tree(s->scene, c.get_ray(u, v), depth, fp->shapes[i], cnt);
                }
        });
    for (auto& t : pool) t.join();
    *out = f.release();
    return RT_OK;
}

rt_status oracle_forest_render_mt(const oracle_forest* f, float* rgb, uint32_t threads) {
    if (!f || !rgb) return RT_ERR_INVALID_ARG;
    if (threads <= 1) return oracle_forest_render(f, rgb);
    std::vector<std::thread> pool;
    const size_t n = f->roots.size();
    for (uint32_t k = 0; k < threads; k++)
        pool.emplace_back([=]() {
            for (size_t i = k; i < n; i += threads) {
                Color col = render_ray_tree(f->roots[i].get(), f->s->scene.ambient).first;
                rgb[3 * i] = col.r; rgb[3 * i + 1] = col.g; rgb[3 * i + 2] = col.b;
            }
        });
    for (auto& t : pool) t.join();
    return RT_OK;
}

rt_status oracle_forest_render(const oracle_forest* f, float* rgb) {
    if (!f || !rgb) return RT_ERR_INVALID_ARG;
    for (size_t k = 0; k < f->roots.size(); k++) {
        Color col = render_ray_tree(f->roots[k].get(), f->s->scene.ambient).first;
        rgb[3 * k] = col.r; rgb[3 * k + 1] = col.g; rgb[3 * k + 2] = col.b;
    }
    return RT_OK;
}

rt_status oracle_forest_render_filter(const oracle_forest* f, const int32_t* ids, uint32_t n_ids, float* rgb) {
    if (!f || !rgb || (n_ids && !ids)) return RT_ERR_INVALID_ARG;
    std::set<int32_t> mutated(ids, ids + n_ids);
    for (size_t k = 0; k < f->roots.size(); k++) {
        bool hit = false;
        for (int32_t id : f->shapes[k])
            if (mutated.count(id)) { hit = true; break; }
        if (!hit) continue;  // the pixel keeps its previous value
        Color col = render_ray_tree(f->roots[k].get(), f->s->scene.ambient).first;
        rgb[3 * k] = col.r; rgb[3 * k + 1] = col.g; rgb[3 * k + 2] = col.b;
    }
    return RT_OK;
}

rt_status oracle_forest_tree_sizes(const oracle_forest* f, uint32_t* sizes) {
    if (!f || !sizes) return RT_ERR_INVALID_ARG;
    for (size_t k = 0; k < f->roots.size(); k++) sizes[k] = tree_size(f->roots[k].get());
    return RT_OK;
}

uint64_t oracle_forest_trees_with(const oracle_forest* f, int32_t id) {  // render_tree.rs:66-71
    uint64_t n = 0;
    if (f)
        for (const auto& st : f->shapes) n += st.count(id) ? 1u : 0u;
    return n;
}

void oracle_forest_destroy(oracle_forest* f) { delete f; }

// Replaces material `index`'s parameters in place (same kind): every shape and every
// cached intersection that holds it sees the new values.
rt_status oracle_scene_set_material(oracle_scene* s, uint32_t index, const rt_material* m) {
    if (!s || !m || index >= s->mats.size()) return RT_ERR_INVALID_ARG;
    Material* cur = s->mats[index].get();
    if (m->kind == RT_MAT_PHONG) {
        Phong* p = dynamic_cast<Phong*>(cur);
        if (!p) return RT_ERR_INVALID_ARG;
        p->ka = cc(m->ambient.color);
        p->kd = cc(m->diffuse.color);
        p->ks = cc(m->specular.color);
        p->power = m->power;
        p->refl = m->reflectivity;
        p->ri = m->refraction_index;
        return RT_OK;
    }
    if (m->kind == RT_MAT_TEXTURE_PHONG) {
        TexturePhong* p = dynamic_cast<TexturePhong*>(cur);
        if (!p) return RT_ERR_INVALID_ARG;
        p->fa = texfun(m->ambient);
        p->fd = texfun(m->diffuse);
        p->fs = texfun(m->specular);
        p->power = m->power;
        p->refl = m->reflectivity;
        p->ri = m->refraction_index;
        return RT_OK;
    }
    return RT_ERR_INVALID_ARG;
}

// f32::powf of the reference (material.rs:211): the platform libm's powf, over arrays
void oracle_powf_batch(const float* x, const float* y, float* out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) out[i] = powf(x[i], y[i]);
}

// the reference's other libm calls (sphere.rs:40-45: f32::atan2 / f32::acos; atanf, which
// atan2f reduces to): fn 1 = atan2f(x[i], y[i]), 2 = acosf(x[i]), 3 = atanf(x[i])
void oracle_libm_batch(int fn, const float* x, const float* y, float* out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++)
        out[i] = fn == 0 ? powf(x[i], y[i]) : fn == 1 ? atan2f(x[i], y[i]) : fn == 2 ? acosf(x[i]) : atanf(x[i]);
}

void oracle_as_u8(const float* rgb, uint64_t n, uint8_t* out) {
    for (uint64_t k = 0; k < n; k++) out[k] = sat_u8(255.f * rgb[k]);
}

void oracle_matrix_identity(float out[16]) { Matrix::identity().store(out); }
void oracle_matrix_scale(float x, float y, float z, float out[16]) { Matrix::scale(x, y, z).store(out); }
void oracle_matrix_translate(float x, float y, float z, float out[16]) { Matrix::translate(x, y, z).store(out); }
void oracle_matrix_rotate_x(float d, float out[16]) { Matrix::rotate_x(d).store(out); }
void oracle_matrix_rotate_y(float d, float out[16]) { Matrix::rotate_y(d).store(out); }
void oracle_matrix_rotate_z(float d, float out[16]) { Matrix::rotate_z(d).store(out); }
void oracle_matrix_mul(const float a[16], const float b[16], float out[16]) {
    Matrix::from(a).mul(Matrix::from(b)).store(out);
}
void oracle_matrix_transpose(const float a[16], float out[16]) { Matrix::from(a).transpose().store(out); }
rt_status oracle_matrix_inverse(const float a[16], float out[16]) {
    Matrix m = Matrix::from(a);
    if (!m.invert()) return RT_ERR_SINGULAR_MATRIX;
    m.store(out);
    return RT_OK;
}
void oracle_matrix_pt_mul(const float m[16], const float p[3], float out[3]) {
    Point3 r = Matrix::from(m).pt_mul(Point3(p[0], p[1], p[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void oracle_matrix_vec3_mul(const float m[16], const float v[3], float out[3]) {
    Vector3 r = Matrix::from(m).vec3_mul(Vector3(v[0], v[1], v[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void oracle_pt_mat_mul(const float p[3], const float m[16], float out[3]) {
    Point3 r = pt_mat_mul(Point3(p[0], p[1], p[2]), Matrix::from(m));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void oracle_vec3_mat_mul(const float v[3], const float m[16], float out[3]) {
    Vector3 r = vec3_mat_mul(Vector3(v[0], v[1], v[2]), Matrix::from(m));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

static std::shared_ptr<Material> white_phong() {
    return std::make_shared<Phong>(WHITE, WHITE, WHITE, 60.f, 1.f, 0.f);
}

void oracle_sphere_intersect(const float transform[16], const float o[3], const float d[3],
                             oracle_hit* out) {
    Sphere s(white_phong());
    s.set_transform(Matrix::from(transform));
    Intersection i;
    bool h = s.intersect(Ray(Point3(o[0], o[1], o[2]), Vector3(d[0], d[1], d[2])), i);
    fill_hit(i, h, out);
}
void oracle_triangle_normal(const float a[3], const float b[3], const float c[3], float out[3]) {
    Triangle t(Point3(a[0], a[1], a[2]), Point3(b[0], b[1], b[2]), Point3(c[0], c[1], c[2]), white_phong());
    out[0] = t.normal.x; out[1] = t.normal.y; out[2] = t.normal.z;
}
void oracle_triangle_intersect(const float a[3], const float b[3], const float c[3],
                               const float o[3], const float d[3], oracle_hit* out) {
    Triangle t(Point3(a[0], a[1], a[2]), Point3(b[0], b[1], b[2]), Point3(c[0], c[1], c[2]), white_phong());
    Intersection i;
    bool h = t.intersect(Ray(Point3(o[0], o[1], o[2]), Vector3(d[0], d[1], d[2])), i);
    fill_hit(i, h, out);
}
void oracle_plane_axes(const float n[3], float u[3], float v[3]) {
    Plane p(Point3(0.f, 0.f, 0.f), Vector3(n[0], n[1], n[2]), white_phong());
    u[0] = p.u.x; u[1] = p.u.y; u[2] = p.u.z;
    v[0] = p.v.x; v[1] = p.v.y; v[2] = p.v.z;
}
void oracle_plane_intersect(const float origin[3], const float n[3], const float transform[16],
                            const float o[3], const float d[3], oracle_hit* out) {
    Plane p(Point3(origin[0], origin[1], origin[2]), Vector3(n[0], n[1], n[2]), white_phong());
    p.set_transform(Matrix::from(transform));
    Intersection i;
    bool h = p.intersect(Ray(Point3(o[0], o[1], o[2]), Vector3(d[0], d[1], d[2])), i);
    fill_hit(i, h, out);
}
void oracle_cube_intersect(const float transform[16], const float o[3], const float d[3],
                           oracle_hit* out) {
    Cube c(white_phong());
    c.set_transform(Matrix::from(transform));
    Intersection i;
    bool h = c.intersect(Ray(Point3(o[0], o[1], o[2]), Vector3(d[0], d[1], d[2])), i);
    fill_hit(i, h, out);
}
void oracle_phong_reflected_energy(const rt_color* a, const rt_color* d, const rt_color* s,
                                   float power, const rt_color* in, const float l[3],
                                   const oracle_hit* h, rt_color* out) {
    Phong p(cc(*a), cc(*d), cc(*s), power, 0.f, 0.f);
    Intersection i;
    i.normal = Vector3(h->normal[0], h->normal[1], h->normal[2]);
    i.eye_dir = Vector3(h->eye_dir[0], h->eye_dir[1], h->eye_dir[2]);
    i.tex_coord = TexCoords(h->tex[0], h->tex[1]);
    Color c = p.get_reflected_energy(cc(*in), Vector3(l[0], l[1], l[2]), i);
    out->r = c.r; out->g = c.g; out->b = c.b;
}
void oracle_checkerboard(float u, float v, rt_color* out) {
    Color c = checkerboard(TexCoords(u, v));
    out->r = c.r; out->g = c.g; out->b = c.b;
}
float oracle_fresnel_reflection(const float l[3], const float n[3], float n1, float n2) {
    return fresnel_reflection(Vector3(l[0], l[1], l[2]), Vector3(n[0], n[1], n[2]), n1, n2);
}

}  // extern "C"
