// rt_build.cpp -- the host half of rt_scene_create (rt_build.hpp).
//
// Validates the flat scene description and runs the scene-build preprocessing the reference
// performs in its constructors and set_transform calls (Matrix::inverse matrix.rs:99-153,
// Plane::new axes plane.rs:22-42, Triangle::new normal triangle.rs:16-39, Cube::new triangles
// cube.rs:21-77), then lays the result out as the device runs of rt_device.hpp: the culling
// hierarchy (rt_bvh.cpp) and its run layout, grazing masks, light buffers (per point light,
// tiered cube maps of record copies) and shape buffers, in one section table.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include <sched.h>

#include "../../include/rt_api.h"
#include "rt_build.hpp"
#include "rt_bvh.hpp"
#include "rt_device.hpp"
#include "rt_tune.hpp"

namespace rtdev {
bool rt_cube_table_check(const float* table);
}  // namespace rtdev

using namespace rtdev;

namespace {

const float EPS = std::numeric_limits<float>::epsilon();

// ---- scene-build math (host).  Same f32 operations, same order as the reference.
struct M4 {
    float m[4][4];
};

// matrix.rs:105-153: Gauss-Jordan; pivot search only when |a_cc| < EPS; a row is
// eliminated only when |coeff| >= EPS; final division by the remaining diagonal.
bool gj_inverse(const float* src, M4& out) {
    float a[4][4], b[4][4];
    std::memcpy(a, src, sizeof(a));
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) b[r][c] = (r == c) ? 1.f : 0.f;
    for (int c = 0; c < 4; c++) {
        if (std::fabs(a[c][c]) < EPS) {
            int piv = c;
            for (int r = 0; r < 4; r++)
                if (std::fabs(a[r][c]) > std::fabs(a[piv][c])) piv = r;
            if (piv == c) return false;  // panic!("Singular Matrix")
            for (int j = 0; j < 4; j++) {
                std::swap(a[piv][j], a[c][j]);
                std::swap(b[piv][j], b[c][j]);
            }
        }
        for (int r = 0; r < 4; r++) {
            if (r == c) continue;
            float k = a[r][c] / a[c][c];
            if (!(std::fabs(k) >= EPS)) continue;
            for (int j = 0; j < 4; j++) {
                a[r][j] -= k * a[c][j];
                b[r][j] -= k * b[c][j];
            }
            a[r][c] = 0.f;
        }
    }
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) b[r][c] /= a[r][r];
    std::memcpy(out.m, b, sizeof(b));
    return true;
}

struct F3 {
    float x, y, z;
};
F3 f3(float x, float y, float z) { return F3{x, y, z}; }
F3 fsub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
F3 fcross(F3 a, F3 b) { return f3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
float flen(F3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
F3 fnorm(F3 a) {
    float l = flen(a);
    return f3(a.x / l, a.y / l, a.z / l);
}
// Triangle::new normal: (v1 - v0) x (v2 - v1), normalised (triangle.rs:25-29)
F3 tri_normal(F3 v0, F3 v1, F3 v2) { return fnorm(fcross(fsub(v1, v0), fsub(v2, v1))); }
F3 vec3_mul(const float* m, F3 v) {  // matrix.rs:240-246 on a row-major 4x4
    return f3(v.x * m[0] + v.y * m[1] + v.z * m[2], v.x * m[4] + v.y * m[5] + v.z * m[6],
              v.x * m[8] + v.y * m[9] + v.z * m[10]);
}

void put4(std::vector<float>& v, float a, float b, float c, float d) {
    v.push_back(a);
    v.push_back(b);
    v.push_back(c);
    v.push_back(d);
}
float keyf(uint32_t k) {
    float f;
    std::memcpy(&f, &k, 4);
    return f;
}

// The 12 triangles of Cube::new in the inner scene's order (cube.rs:21-69):
// tf1 tf2 tk1 tk2 tr1 tr2 tl1 tl2 tt1 tt2 tb1 tb2.
void cube_triangles(std::vector<float>& out) {
    const F3 v0 = f3(0.5f, 0.5f, -0.5f), v1 = f3(0.5f, -0.5f, -0.5f), v2 = f3(-0.5f, -0.5f, -0.5f),
             v3 = f3(-0.5f, 0.5f, -0.5f), v4 = f3(0.5f, 0.5f, 0.5f), v5 = f3(-0.5f, 0.5f, 0.5f),
             v6 = f3(-0.5f, -0.5f, 0.5f), v7 = f3(0.5f, -0.5f, 0.5f);
    const F3 tris[12][3] = {{v1, v2, v3}, {v0, v1, v3}, {v7, v5, v4}, {v5, v7, v6},
                            {v0, v4, v7}, {v7, v1, v0}, {v5, v3, v6}, {v6, v3, v2},
                            {v5, v4, v0}, {v0, v3, v5}, {v1, v7, v6}, {v6, v2, v1}};
    for (int k = 0; k < 12; k++) {
        F3 a = tris[k][0], b = tris[k][1], c = tris[k][2];
        F3 e1 = fsub(b, a), e2 = fsub(c, a), n = tri_normal(a, b, c);
        put4(out, a.x, a.y, a.z, 0.f);
        put4(out, e1.x, e1.y, e1.z, 0.f);
        put4(out, e2.x, e2.y, e2.z, 0.f);
        put4(out, n.x, n.y, n.z, 0.f);
    }
}

// rt_material -> device record (material.rs: Phong / TexturePhong with a closed set of
// texture programs)
// The combine pass skips a shadowed point light of a node (rt_wavefront.hip light_sum)
// only when its term f * ((l.n * 0) * kd + (pw * 0) * ks) is exactly +-0: the Schlick r0
// and the fresnel factor finite for either side of the surface (n1 + n2 = 1 + ri != 0,
// |1 - r0| x (1 + |n|)^5 finite for |n| <= 1e3), (m.h)^power finite (power in [0, 1e6] and
// power x ln(nmax (1 + 1e-5)) < 80, nmax = the scene's largest hit-normal length: planes
// shade with the unnormalised transform * normal, plane.rs:75, so m.h can exceed 1 and
// (m.h)^power overflow to inf, where the reference's inf * BLACK is NaN, material.rs:211),
// finite diffuse / specular colours.
bool dark_zero(const rt_material& m, double nmax) {
    auto finite_tex = [](const rt_texture& t) {
        return t.kind == RT_TEX_CHECKERBOARD ||
               (std::isfinite(t.color.r) && std::isfinite(t.color.g) && std::isfinite(t.color.b));
    };
    const float ri = m.refraction_index;
    if (!(std::isfinite(m.power) && m.power >= 0.f && m.power <= 1e6f && std::isfinite(ri))) return false;
    if (!(std::isfinite(nmax) && (double)m.power * std::log(std::max(1.0, nmax) * (1.0 + 1e-5)) < 80.0)) return false;
    for (int entering = 0; entering < 2; entering++) {
        const float n1 = entering ? 1.f : ri, n2 = entering ? ri : 1.f;
        const float q = (n1 - n2) / (n1 + n2), r0 = q * q;
        if (!std::isfinite(q) || !std::isfinite(r0) || !(std::fabs(1.0 - (double)r0) * 1.01e15 < 1e37)) return false;
    }
    return finite_tex(m.diffuse) && finite_tex(m.specular);
}

rt_status mat_rec(const rt_material& m, MatRec& M, double nmax) {
    if (m.kind != RT_MAT_PHONG && m.kind != RT_MAT_TEXTURE_PHONG) return RT_ERR_INVALID_ARG;
    const rt_texture* tx[3] = {&m.ambient, &m.diffuse, &m.specular};
    for (int k = 0; k < 3; k++) {
        if (tx[k]->kind != RT_TEX_CONST && tx[k]->kind != RT_TEX_CHECKERBOARD) return RT_ERR_INVALID_ARG;
        // Phong ignores texture programs: its colours are constants (material.rs:55-65)
        if (m.kind == RT_MAT_PHONG && tx[k]->kind != RT_TEX_CONST) return RT_ERR_INVALID_ARG;
    }
    std::memset(&M, 0, sizeof(M));
    M.kind = m.kind;
    M.dark_zero = dark_zero(m, nmax) ? 1 : 0;
    M.power = m.power;
    M.reflectivity = m.reflectivity;
    M.refraction_index = m.refraction_index;
    M.ambient = TexRec{m.ambient.kind, m.ambient.color.r, m.ambient.color.g, m.ambient.color.b};
    M.diffuse = TexRec{m.diffuse.kind, m.diffuse.color.r, m.diffuse.color.g, m.diffuse.color.b};
    M.specular = TexRec{m.specular.kind, m.specular.color.r, m.specular.color.g, m.specular.color.b};
    return RT_OK;
}

// ---- culling hierarchy (rt_bvh.hpp) and the run layout --------------------------------
struct SphIn {
    float inv[12];
    float key;
    bool diag;
};
struct TriIn {
    F3 v[3], e1, e2;
    float key;
};
struct CubeIn {
    float inv[12];
    float key;
};

// A hierarchy primitive as the light buffers see it: bounding ball and the run record
// that tests it (LB_* type << 30 | record index).
enum : uint32_t { LB_DSPH = 0, LB_GSPH = 1, LB_TRI = 2, LB_CUBE = 3 };
constexpr size_t RUN_WIDTH[4] = {16, 16, 24, 16};  // floats per record of each run array
struct LbPrim {
    double c[3], r;
    uint32_t code;
    uint32_t shape;  // insertion index of the primitive's shape (a pair record: this member's)
    double h3;       // this primitive's own bound h_P(D) at D = 3 R (+ the slab terms): how far
                     // from it a hit it reports can lie, for any origin within 3 R of the centre
    double p2, p1, p0;  // ... as the polynomial h_P(D) = ((p2 D + p1) D + p0) (1 + 1e-6)
    double h_at(double D) const { return ((p2 * D + p1) * D + p0) * (1 + 1e-6); }
};

struct RunLayout {
    std::vector<float> dsph, gsph, tri, cube, nodes, graze_blk, graze_tri;
    // grazing pass by direction cell: per graze pair its two normals / sin(phi_T)
    // {nAx nBx nAy nBy} {nAz nBz - -}; per cell of a res x res cube map of directions a
    // bitmask (graze_words words) of the pairs some direction in the cell can graze
    std::vector<float> graze_pn;
    std::vector<uint32_t> graze_mask;
    uint32_t graze_res = 0, graze_words = 0;
    std::vector<uint32_t> leaves;
    std::vector<LbPrim> lb_prims;  // every hierarchy primitive (light buffers)
    // Record copies that follow a run array's own records in the device image: the light
    // buffers' cells, then the shape buffers.  Kept apart (never concatenated on the host:
    // the upload places each piece); lb is filled in parallel, uninitialised until then.
    struct Ext {
        std::unique_ptr<float[]> lb;
        size_t lb_floats = 0;
        std::vector<float> sb;
    };
    Ext ext[4];  // LB_DSPH, LB_GSPH, LB_TRI, LB_CUBE
    uint32_t root = BVH_LEAF;
    bool use = false;
    int n_dsph_bvh = 0, n_gsph_bvh = 0, n_tri_bvh = 0, n_cube_bvh = 0;
    float c[3] = {0, 0, 0}, r = 0, g2 = 0, g1 = 0, g0 = 0, m1 = 0, m0 = 0;
};


// Safety factors over the largest ratios tools/cull_bounds_check.py measures for each
// bound (sphere 0.43, cube 1.83; triangles: the reported hit point's distance
// rho eps (|o - v0| + |e|max + |o| + |v0|) / (sin(alpha) sin(phi)) with rho <= 0.6 for
// sin(phi) < 0.1 and rho / sin(phi) <= 1.3 above).
constexpr double SAFETY_SPHERE = 4.0, SAFETY_CUBE = 32.0, SAFETY_TRI = 4.0, TRI_STEEP = 10.0,
                 SAFETY_SLAB = 4.0;
constexpr double MAX_COND = 100.0;          // sigma_max(L) sigma_max(A) above it: linear pass
constexpr double MIN_SIN_ALPHA = 0.02;      // sliver triangles: linear pass
const double FEPS = (double)std::numeric_limits<float>::epsilon();

// A hierarchy triangle's grazing threshold sin(phi_T) = GRAZE_K / sin(alpha), clamped:
// rays meeting its plane at sin(phi) < 1.01 sin(phi_T) go to the grazing pass; the
// rest are covered by its box grown by SAFETY_TRI eps (...) / (sin(alpha) sin(phi_T)).
// GRAZE_K trades the grazing band's width against that growth (RT_GRAZE_K overrides).
constexpr double GRAZE_MIN = 2e-4, GRAZE_MAX = 0.05;
double graze_sin(double sin_a, double k) { return std::min(GRAZE_MAX, std::max(GRAZE_MIN, k / sin_a)); }

float down_f(double x) {
    float f = (float)x;
    return ((double)f > x) ? std::nextafter(f, -std::numeric_limits<float>::infinity()) : f;
}
float up_f(double x) {
    float f = (float)x;
    return ((double)f < x) ? std::nextafter(f, std::numeric_limits<float>::infinity()) : f;
}

struct Geo {          // f64 view of one hierarchy primitive
    double lo[3], hi[3], c[3], r;   // box, bounding ball
    double a2, a1, a0;              // inflation coefficients (D-polynomial)
};

// upper bound of the spectral norm: sqrt(|M^T M|_inf) >= sigma_max (exact for
// rotation x diagonal matrices)
double sig_up(const double m[3][3]) {
    double best = 0;
    for (int i = 0; i < 3; i++) {
        double row = 0;
        for (int j = 0; j < 3; j++) {
            double g = 0;
            for (int k = 0; k < 3; k++) g += m[k][i] * m[k][j];
            row += std::fabs(g);
        }
        best = std::max(best, row);
    }
    return std::sqrt(best) * (1 + 1e-9);
}
bool inv3(const double m[3][3], double o[3][3]) {
    double c00 = m[1][1] * m[2][2] - m[1][2] * m[2][1], c01 = m[1][2] * m[2][0] - m[1][0] * m[2][2],
           c02 = m[1][0] * m[2][1] - m[1][1] * m[2][0];
    double det = m[0][0] * c00 + m[0][1] * c01 + m[0][2] * c02;
    if (!(std::fabs(det) > 0) || !std::isfinite(det)) return false;
    double id = 1.0 / det;
    o[0][0] = c00 * id;
    o[1][0] = c01 * id;
    o[2][0] = c02 * id;
    o[0][1] = (m[0][2] * m[2][1] - m[0][1] * m[2][2]) * id;
    o[1][1] = (m[0][0] * m[2][2] - m[0][2] * m[2][0]) * id;
    o[2][1] = (m[0][1] * m[2][0] - m[0][0] * m[2][1]) * id;
    o[0][2] = (m[0][1] * m[1][2] - m[0][2] * m[1][1]) * id;
    o[1][2] = (m[0][2] * m[1][0] - m[0][0] * m[1][2]) * id;
    o[2][2] = (m[0][0] * m[1][1] - m[0][1] * m[1][0]) * id;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            if (!std::isfinite(o[i][j])) return false;
    return true;
}

// Sphere (cube == false) or cube: E = { A u + c : |u| <= 1 } (resp. u in [-1/2, 1/2]^3)
// with A = L^-1, c = -A s for the stored f32 inverse (L | s).  Returns false when the
// transform is too ill-conditioned for the hierarchy.
bool geo_affine(const float* inv, bool is_cube, Geo& g, double& sigL, double& snorm, double& sigA) {
    double L[3][3], A[3][3], s[3];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) L[i][j] = inv[i * 4 + j];
        s[i] = inv[i * 4 + 3];
    }
    if (!inv3(L, A)) return false;
    sigL = sig_up(L);
    sigA = sig_up(A);
    snorm = std::sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    if (!(sigL * sigA <= MAX_COND) || !std::isfinite(snorm)) return false;
    for (int i = 0; i < 3; i++) {
        g.c[i] = -(A[i][0] * s[0] + A[i][1] * s[1] + A[i][2] * s[2]);
        double h = is_cube ? 0.5 * (std::fabs(A[i][0]) + std::fabs(A[i][1]) + std::fabs(A[i][2]))
                           : std::sqrt(A[i][0] * A[i][0] + A[i][1] * A[i][1] + A[i][2] * A[i][2]);
        h = h * (1 + 1e-9) + 1e-30;
        g.lo[i] = g.c[i] - h;
        g.hi[i] = g.c[i] + h;
    }
    g.r = (is_cube ? 0.5 * std::sqrt(3.0) : 1.0) * sigA * (1 + 1e-9);
    return std::isfinite(g.r);
}

void emit_dsph_pair(std::vector<float>& v, const SphIn& A, const SphIn& B) {
    put4(v, A.inv[0], B.inv[0], A.inv[5], B.inv[5]);
    put4(v, A.inv[10], B.inv[10], A.inv[3], B.inv[3]);
    put4(v, A.inv[7], B.inv[7], A.inv[11], B.inv[11]);
    put4(v, A.key, B.key, 0.f, 0.f);
}
void emit_gsph(std::vector<float>& v, const SphIn& A) {  // a diag sphere's rows hold its zeros
    for (int r = 0; r < 3; r++) put4(v, A.inv[r * 4], A.inv[r * 4 + 1], A.inv[r * 4 + 2], A.inv[r * 4 + 3]);
    put4(v, A.key, 0.f, 0.f, 0.f);
}
// loose triangle pair; B == nullptr pads with a degenerate triangle (e1 = e2 = 0 ->
// det = 0 -> |det| < EPS: never a hit)
void emit_tri_pair(std::vector<float>& v, const TriIn& A, const TriIn* Bp) {
    TriIn pad;
    pad.v[0] = pad.e1 = pad.e2 = f3(0, 0, 0);
    pad.key = keyf(0xFFFFFFF0u);
    const TriIn& B = Bp ? *Bp : pad;
    put4(v, A.v[0].x, B.v[0].x, A.v[0].y, B.v[0].y);
    put4(v, A.v[0].z, B.v[0].z, A.e1.x, B.e1.x);
    put4(v, A.e1.y, B.e1.y, A.e1.z, B.e1.z);
    put4(v, A.e2.x, B.e2.x, A.e2.y, B.e2.y);
    put4(v, A.e2.z, B.e2.z, A.key, B.key);
    put4(v, 0.f, 0.f, 0.f, 0.f);
}
F3 unit_normal(const TriIn& t) {
    double a[3] = {t.v[0].x, t.v[0].y, t.v[0].z}, b[3] = {t.v[1].x, t.v[1].y, t.v[1].z},
           c[3] = {t.v[2].x, t.v[2].y, t.v[2].z};
    double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
    double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    double l = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    return f3((float)(n[0] / l), (float)(n[1] / l), (float)(n[2] / l));
}
void emit_cube(std::vector<float>& v, const CubeIn& A, float lf, float sn) {
    for (int r = 0; r < 3; r++) put4(v, A.inv[r * 4], A.inv[r * 4 + 1], A.inv[r * 4 + 2], A.inv[r * 4 + 3]);
    put4(v, A.key, lf, sn, 0.f);
}

// Grazing pass data (rt_scan.hpp graze_pass): the hierarchy's triangles ordered by
// normal direction (sign-free) in blocks of 8, each with a cone {axis, s^2}: a ray with
// (d.axis)^2 > s^2 |d|^2 meets every plane of the block at sin(phi) > 1.01 sin(phi_T).
// The normals are stored divided by sin(phi_T), so "(d.n')^2 < 1.0201 |d|^2" is the
// per-triangle grazing test.  Block: {ax ay az s^2} {n'x0-3} {n'x4-7} {n'y0-3} {n'y4-7}
// {n'z0-3} {n'z4-7} {-}; its triangles as 4 pairs in graze_tri.
static void lb_face_dir(int f, double a, double b, double out[3]);

void build_graze(const std::vector<TriIn>& tris, const std::vector<char>& in_tri, const std::vector<double>& gsin,
                 RunLayout& L, const Tune& tn) {
    struct G {
        const TriIn* t;
        double n[3];
        uint32_t code;
        double s;
    };
    std::vector<G> g;
    for (size_t i = 0; i < tris.size(); i++) {
        if (!in_tri[i]) continue;
        F3 u = unit_normal(tris[i]);
        double n[3] = {u.x, u.y, u.z};
        int big = 0;
        for (int k = 1; k < 3; k++)
            if (std::fabs(n[k]) > std::fabs(n[big])) big = k;
        if (n[big] < 0)
            for (double& x : n) x = -x;
        // octahedral map of the (sign-free) normal -> 2 x 8 bits, Morton order
        double l1 = std::fabs(n[0]) + std::fabs(n[1]) + std::fabs(n[2]);
        double px = n[0] / l1, py = n[1] / l1;
        if (n[2] < 0) {
            double qx = (1 - std::fabs(py)) * (px >= 0 ? 1 : -1), qy = (1 - std::fabs(px)) * (py >= 0 ? 1 : -1);
            px = qx;
            py = qy;
        }
        uint32_t ix = (uint32_t)std::min(255.0, std::max(0.0, (px * 0.5 + 0.5) * 256.0));
        uint32_t iy = (uint32_t)std::min(255.0, std::max(0.0, (py * 0.5 + 0.5) * 256.0));
        uint32_t code = 0;
        for (int b = 0; b < 8; b++) code |= (((ix >> b) & 1u) << (2 * b)) | (((iy >> b) & 1u) << (2 * b + 1));
        g.push_back(G{&tris[i], {n[0], n[1], n[2]}, code, gsin[i]});
    }
    std::stable_sort(g.begin(), g.end(), [](const G& a, const G& b) { return a.code < b.code; });
    for (size_t b0 = 0; b0 < g.size(); b0 += 8) {
        size_t b1 = std::min(g.size(), b0 + 8);
        double smax = 0;
        for (size_t i = b0; i < b1; i++) smax = std::max(smax, g[i].s);
        const double phi = std::asin(std::min(1.0, 1.01 * smax)) + 1e-4;
        double a[3] = {0, 0, 0};
        for (size_t i = b0; i < b1; i++)
            for (int k = 0; k < 3; k++) a[k] += g[i].n[k];
        double la = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        double s2 = 1.0;  // no usable cone: always test the normals
        if (la > 1e-6) {
            for (double& x : a) x /= la;
            double cmin = 1.0;
            for (size_t i = b0; i < b1; i++)
                cmin = std::min(cmin, std::fabs(a[0] * g[i].n[0] + a[1] * g[i].n[1] + a[2] * g[i].n[2]));
            double theta = std::acos(std::min(1.0, cmin)) + 1e-4;
            if (theta + phi < 1.5707) s2 = std::pow(std::sin(theta + phi), 2) * (1 + 1e-4);
        } else {
            a[0] = 1;
            a[1] = a[2] = 0;
        }
        float nx[8], ny[8], nz[8];
        for (int k = 0; k < 8; k++) {
            if (b0 + k < b1) {
                F3 u = unit_normal(*g[b0 + k].t);
                double is = 1.0 / g[b0 + k].s;
                nx[k] = (float)(u.x * is);
                ny[k] = (float)(u.y * is);
                nz[k] = (float)(u.z * is);
            } else {  // padding: never grazes (and its pair slot is a degenerate triangle)
                nx[k] = ny[k] = nz[k] = 1e18f;
            }
        }
        put4(L.graze_blk, (float)a[0], (float)a[1], (float)a[2], up_f(std::min(1.0, s2)));
        put4(L.graze_blk, nx[0], nx[1], nx[2], nx[3]);
        put4(L.graze_blk, nx[4], nx[5], nx[6], nx[7]);
        put4(L.graze_blk, ny[0], ny[1], ny[2], ny[3]);
        put4(L.graze_blk, ny[4], ny[5], ny[6], ny[7]);
        put4(L.graze_blk, nz[0], nz[1], nz[2], nz[3]);
        put4(L.graze_blk, nz[4], nz[5], nz[6], nz[7]);
        put4(L.graze_blk, 0.f, 0.f, 0.f, 0.f);
        for (int k = 0; k < 8; k += 2)  // the pairs' normals for the direction-cell path
            put4(L.graze_pn, nx[k], nx[k + 1], ny[k], ny[k + 1]), put4(L.graze_pn, nz[k], nz[k + 1], 0.f, 0.f);
        for (int k = 0; k < 8; k += 2) {
            const TriIn* A = (b0 + k < b1) ? g[b0 + k].t : nullptr;
            const TriIn* B = (b0 + k + 1 < b1) ? g[b0 + k + 1].t : nullptr;
            if (A) emit_tri_pair(L.graze_tri, *A, B);
            else {
                TriIn pad;
                pad.v[0] = pad.e1 = pad.e2 = f3(0, 0, 0);
                pad.key = keyf(0xFFFFFFF0u);
                emit_tri_pair(L.graze_tri, pad, nullptr);
            }
        }
    }
    // direction cells (RT_GRAZE_RES per face side, 0: cone path only): pair p is set in
    // a cell when a direction within the cell's angular radius rc (+1e-4) of its centre
    // can meet one of its triangles' planes at sin(phi) < 1.01 sin(phi_T): |c.n| <=
    // sin(asin(1.01 s) + rc + 1e-4).  Exact superset of the per-lane test.
    const int R = tn.graze_res;
    const size_t npairs = L.graze_pn.size() / 8;
    if (R > 0 && R <= 256 && npairs > 0 && npairs <= 256) {
        const uint32_t W = (uint32_t)((npairs + 31) / 32);
        L.graze_res = (uint32_t)R;
        L.graze_words = W;
        L.graze_mask.assign((size_t)6 * R * R * W, 0u);
        // per pair: unit normals and band limits
        std::vector<double> pn(npairs * 6), plim(npairs * 2);
        for (size_t p = 0; p < npairs; p++)
            for (int k = 0; k < 2; k++) {
                const size_t gi = 2 * p + k;  // index into g (blocks of 8, pairs in order)
                if (gi >= g.size()) {
                    plim[2 * p + k] = -1.0;  // padding
                    continue;
                }
                for (int c = 0; c < 3; c++) pn[6 * p + 3 * k + c] = g[gi].n[c];
                plim[2 * p + k] = std::asin(std::min(1.0, 1.01 * g[gi].s));
            }
        for (int f = 0; f < 6; f++)
            for (int j = 0; j < R; j++)
                for (int i = 0; i < R; i++) {
                    const double a0 = -1.0 + 2.0 * i / R, a1 = -1.0 + 2.0 * (i + 1) / R;
                    const double b0 = -1.0 + 2.0 * j / R, b1 = -1.0 + 2.0 * (j + 1) / R;
                    double m[3], q[3];
                    lb_face_dir(f, 0.5 * (a0 + a1), 0.5 * (b0 + b1), m);
                    double rc = 0;
                    for (double aa : {a0, a1})
                        for (double bb : {b0, b1}) {
                            lb_face_dir(f, aa, bb, q);
                            rc = std::max(rc, std::acos(std::min(1.0, m[0] * q[0] + m[1] * q[1] + m[2] * q[2])));
                        }
                    rc = rc * 1.01 + 1e-6;
                    uint32_t* mw = &L.graze_mask[(((size_t)f * R + j) * R + i) * W];
                    for (size_t p = 0; p < npairs; p++)
                        for (int k = 0; k < 2; k++) {
                            if (plim[2 * p + k] < 0) continue;
                            const double* n = &pn[6 * p + 3 * k];
                            const double cn = std::fabs(m[0] * n[0] + m[1] * n[1] + m[2] * n[2]);
                            const double ang = plim[2 * p + k] + rc + 1e-4;
                            if (ang >= 1.5707963 || cn <= std::sin(ang)) mw[p / 32] |= 1u << (p % 32);
                        }
                }
    }
}

// Lays out the runs: hierarchy primitives leaf by leaf, then the linear rest.  Within
// a leaf diag spheres pair up (an odd one joins the general run), triangles pair up.
// Light buffers (shadow rays; DESIGN.md "Light buffers").  Per point light, a cube map
// of R x R cells per face over the directions from the light; cell c lists every
// hierarchy record with a primitive whose ball, grown by the hierarchy's bound h(D_max),
// subtends (from the light, plus LB_MU) a direction inside the cell -- sorted by the
// ball's nearest distance to the light.  A shadow ray toward the light whose origin has
// D <= D_max and distance to the light <= LB_LMAX can only get a hit that shadows from a
// primitive listed in the cell of its direction: such a hit point X lies on the ray
// within h(D) of the primitive, between the origin and the light, and the direction
// lpos -> X is within |delta d| (1 + Lambda / rho) <= LB_MU / 2 of -d (|delta d| <= 1e-6,
// the rounding of d = norm(lpos - o); |X - lpos| >= rho = LB_RHO since no grown ball
// comes nearer the light: else the light gets no buffer).
constexpr double LB_MU = 2e-3, LB_RHO = 0.05;  // LB_LMAX: RT_LB_LMAX (rt_device.hpp)

// Each cell becomes a leaf record of the hierarchy's leaf table whose runs are copies
// of the listed records (appended to the run arrays after the linear rest), so a cell is
// tested exactly like a leaf (prefetching run loops).
struct LightBuffers {
    uint32_t res = 0;
    uint32_t tiers = 0;             // tier t: origins with D <= dmax 2^t (cells at base + t 6 res^2)
    std::vector<uint32_t> base;     // per light: leaf index of its first cell, or ~0 (no buffer)
    float dmax = 0.f;
};

// the cube-map cell of direction v (same face / axis conventions as rt_scan.hpp lb_cell)
static void lb_face_dir(int f, double a, double b, double out[3]) {
    const int k = f >> 1;
    const double s = (f & 1) ? -1.0 : 1.0;
    const int u = k == 0 ? 1 : 0, v = k == 2 ? 1 : 2;
    out[k] = s;
    out[u] = a;
    out[v] = b;
    const double l = std::sqrt(out[0] * out[0] + out[1] * out[1] + out[2] * out[2]);
    for (int i = 0; i < 3; i++) out[i] /= l;
}

// Host threads the scene build may use: Tune::build_threads, or the CPUs of the process's
// affinity mask capped by its cgroup CPU quota (a container may see 256 CPUs and be granted
// 16), at most 32.
int build_thread_count(const Tune& T) {
    if (T.build_threads > 0) return T.build_threads;
    int n = 1;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::max(1, CPU_COUNT(&set));
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {  // cgroup v2: "quota period" or "max period"
        char q[32] = {0};
        long long period = 0;
        if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0) {
            const long long quota = std::atoll(q);
            if (quota > 0) n = std::min<long long>(n, std::max(1LL, (quota + period - 1) / period));
        }
        std::fclose(f);
    }
    return std::min(n, 32);
}

// Runs f(0 .. n_jobs - 1) over up to `threads` host threads (the calling thread included).
template <class F>
void parallel_jobs(int n_jobs, int threads, F&& f) {
    threads = std::max(1, std::min(threads, n_jobs));
    std::atomic<int> next{0};
    auto worker = [&]() {
        for (int j; (j = next.fetch_add(1)) < n_jobs;) f(j);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
}

// One (light, tier) job of build_light_buffers: the cone of every hierarchy primitive's grown
// ball seen from the light (nearest first), then per cell the records whose cone meets the
// cell (a pair record listed once) and, per cell and record type, the place of their copies.
struct LbJob {
    uint32_t li = 0;
    int tier = 0;
    struct Cone {
        double u[3], alpha, ca, sa, near;
        uint32_t code;
        int prev_same;  // the previous cone (nearest-first order) of the same record, or -1
        uint8_t faces;  // the cube-map faces the cone may meet
        bool all;       // its record is in the tier's all-cell leaf instead of cell lists
    };
    std::vector<Cone> cones;
    struct Ent {
        uint32_t code;
        float near;  // down-rounded nearest distance to the light (0 without the reach cut)
    };
    std::vector<std::vector<std::pair<uint32_t, Ent>>> chunk_hits;  // (cell, entry) per cone chunk
    std::vector<uint32_t> cell_start;  // [nc + 1] into `ent` (entries grouped by cell)
    std::vector<Ent> ent;
    std::vector<uint32_t> cell_first;  // [4 nc]: per cell and type its first copy (job-relative)
    // the tier's all-cell leaf: every record one of whose cones covers every direction (its
    // grown ball within LB_RHO of the light), once, nearest first -- instead of a copy in each
    // of the 6 res^2 cells
    std::vector<Ent> all_ent;
    size_t all_first[4] = {0, 0, 0, 0};  // its first copy per type (job-relative)
    uint32_t cell_leaf = 0, all_leaf = 0;  // leaf indices: the tier's first cell, the all-cell leaf
    size_t count[4] = {0, 0, 0, 0};  // copies per record type
    size_t first[4] = {0, 0, 0, 0};  // the job's first copy in each run array
};

void build_light_buffers(RunLayout& L, const std::vector<LightRec>& lights, LightBuffers& B, const Tune& T) {
    const int R = T.lb_res;  // cells per face side; 0: no light buffers (A/B)
    const bool reach_cut = T.lb_reach != 0;  // 0: runs are never cut at the reach (A/B)
    B.base.assign(lights.size(), 0xFFFFFFFFu);
    if (!L.use || R <= 0 || R > 1024 || L.lb_prims.empty()) return;
    B.res = (uint32_t)R;
    // origins farther than D_max from the scene ball's centre (+ R) use the hierarchy walk
    const double dmax = T.lb_dmax_k * (double)L.r;  // tier 0 (Tune::lb_dmax_k, default 3)
    B.dmax = down_f(dmax);
    // cell centres and angular radii (max angle to a corner, +1%)
    const int nc = 6 * R * R;
    std::vector<double> cdir(3 * (size_t)nc), ccos(nc), csin(nc), crad(nc);
    for (int f = 0; f < 6; f++)
        for (int j = 0; j < R; j++)
            for (int i = 0; i < R; i++) {
                const size_t c = ((size_t)f * R + j) * R + i;
                const double a0 = -1.0 + 2.0 * i / R, a1 = -1.0 + 2.0 * (i + 1) / R;
                const double b0 = -1.0 + 2.0 * j / R, b1 = -1.0 + 2.0 * (j + 1) / R;
                double m[3], q[3];
                lb_face_dir(f, 0.5 * (a0 + a1), 0.5 * (b0 + b1), m);
                double rad = 0;
                for (double a : {a0, a1})
                    for (double b : {b0, b1}) {
                        lb_face_dir(f, a, b, q);
                        rad = std::max(rad, std::acos(std::min(1.0, m[0] * q[0] + m[1] * q[1] + m[2] * q[2])));
                    }
                rad = rad * 1.01 + 1e-6;
                for (int k = 0; k < 3; k++) cdir[3 * c + k] = m[k];
                ccos[c] = std::cos(rad);
                csin[c] = std::sin(rad);
                crad[c] = rad;
            }
    const double PI = 3.14159265358979323846;
    const double FACE_HALF = 0.9556;  // a face's directions lie within 54.75 deg of its axis
    // blocks of up to 8 x 8 cells: a direction and an angle brad that exceeds the angle to
    // every cell centre of the block plus that cell's radius.  A cone whose axis lies more
    // than alpha + brad + 1e-4 rad from the block's direction meets none of its cells (the
    // cell test below fails for each by far more than its 1e-12 slack), so the block is skipped
    const int BS = 8, NB = (R + BS - 1) / BS;
    std::vector<double> bdir(3 * (size_t)6 * NB * NB), brad((size_t)6 * NB * NB);
    for (int f = 0; f < 6; f++)
        for (int bj = 0; bj < NB; bj++)
            for (int bi = 0; bi < NB; bi++) {
                const size_t b = ((size_t)f * NB + bj) * NB + bi;
                const int i0 = bi * BS, i1 = std::min(R, i0 + BS), j0 = bj * BS, j1 = std::min(R, j0 + BS);
                double m[3];
                lb_face_dir(f, -1.0 + (double)(i0 + i1) / R, -1.0 + (double)(j0 + j1) / R, m);
                double rad = 0;
                for (int j = j0; j < j1; j++)
                    for (int i = i0; i < i1; i++) {
                        const size_t c = ((size_t)f * R + j) * R + i;
                        const double dt = m[0] * cdir[3 * c] + m[1] * cdir[3 * c + 1] + m[2] * cdir[3 * c + 2];
                        rad = std::max(rad, std::acos(std::max(-1.0, std::min(1.0, dt))) + crad[c]);
                    }
                for (int k = 0; k < 3; k++) bdir[3 * b + k] = m[k];
                brad[b] = rad;
            }
    // Tier t serves origins with D <= dmax 2^t and a light within LB_LMAX 2^t (the device
    // compares with down_f(dmax) 2^t and RT_LB_LMAX^2 4^t): every primitive's ball grown by
    // its own bound at that reach (at most the hierarchy's), its cone by LB_MU 2^t (the
    // direction error |delta d| (1 + Lambda / rho) doubles with Lambda's limit).  Tiers beyond
    // the first catch the walk's costliest rays -- far origins, whose bound grows as D^2
    // (DESIGN.md "Where the shadow scan's cycles go").
    auto hmax_at = [&](double dm) { return ((double)L.g2 * dm + (double)L.g1) * dm + (double)L.g0; };
    auto grown = [&](const LbPrim& p, double dm) { return (p.r + std::min(p.h_at(dm), hmax_at(dm))) * (1 + 1e-6); };
    auto light_ok = [&](const double lp[3], double dm) {  // no grown ball comes within LB_RHO of the light
        for (const LbPrim& p : L.lb_prims) {
            const double w[3] = {p.c[0] - lp[0], p.c[1] - lp[1], p.c[2] - lp[2]};
            if (!(std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]) - grown(p, dm) >= LB_RHO)) return false;
        }
        return true;
    };
    // per light: the most tiers (<= Tune::lb_tiers) whose grown balls all keep LB_RHO from it
    const int max_tiers = std::max(1, std::min(7, T.lb_tiers));
    // Tune::lb_near_all: tier 0 as before, and every further tier: a record whose grown ball
    // comes within LB_RHO of the light goes into every cell of that tier (a hit on it may lie
    // in any direction from the light); the others keep the direction bound with rho = LB_RHO
    auto tiers_of = [&](const double lp[3]) {
        if (T.lb_near_all) return light_ok(lp, dmax) ? max_tiers : 0;
        int n = 0;
        while (n < max_tiers && light_ok(lp, dmax * (double)(1 << n))) n++;
        return n;
    };
    B.tiers = 0;
#if RT_DIAG
    if (std::getenv("RT_LB_DEBUG"))
        for (const LightRec& lr : lights) {
            const double lp[3] = {lr.px, lr.py, lr.pz};
            int ok_t = 0;
            while (ok_t < 7 && light_ok(lp, dmax * (double)(1 << ok_t))) ok_t++;
            double near = 1e30;
            for (const LbPrim& p : L.lb_prims) {
                const double w[3] = {p.c[0] - lp[0], p.c[1] - lp[1], p.c[2] - lp[2]};
                near = std::min(near, std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]) - p.r);
            }
            std::fprintf(stderr, "light (%g %g %g): tiers it supports %d (nearest ball surface %g); R %g\n",
                         lp[0], lp[1], lp[2], ok_t, near, (double)L.r);
        }
#endif
    // the jobs: every tier of every light that gets a buffer, in light then tier order (the
    // order their cells take in the leaf table and their copies in the run arrays)
    std::vector<LbJob> jobs;
    uint32_t next_leaf = (uint32_t)(L.leaves.size() / 8);
    for (size_t li = 0; li < lights.size(); li++) {
        if (lights[li].kind != RT_LIGHT_POINT) continue;
        const double lp[3] = {lights[li].px, lights[li].py, lights[li].pz};
        const int tiers = tiers_of(lp);
        if (tiers == 0) continue;  // a primitive (nearly) at the light: no buffer
        if (next_leaf >= (1u << 28)) continue;  // (the tier count sits in LightRec::lb_base's top bits)
        B.base[li] = next_leaf | ((uint32_t)tiers << 28);
        B.tiers = std::max(B.tiers, (uint32_t)tiers);
        // a light's leaves: tier 0's cells, tier 1's, ..., then one all-cell leaf per tier
        for (int t = 0; t < tiers; t++) {
            LbJob jb;
            jb.li = (uint32_t)li;
            jb.tier = t;
            jb.cell_leaf = next_leaf + (uint32_t)(t * nc);
            jb.all_leaf = next_leaf + (uint32_t)(tiers * nc + t);
            jobs.push_back(std::move(jb));
        }
        next_leaf += (uint32_t)(tiers * nc + tiers);
    }
    if (jobs.empty()) return;
    const int threads = build_thread_count(T);
    // (1) per job: the cones, nearest first, their faces and same-record links
    parallel_jobs((int)jobs.size(), threads, [&](int ji) {
        LbJob& jb = jobs[ji];
        const double lp[3] = {lights[jb.li].px, lights[jb.li].py, lights[jb.li].pz};
        const int t = jb.tier;
        const double dm = dmax * (double)(1 << t);
        std::vector<LbJob::Cone>& cones = jb.cones;
        cones.reserve(L.lb_prims.size());
        for (const LbPrim& p : L.lb_prims) {
            double w[3] = {p.c[0] - lp[0], p.c[1] - lp[1], p.c[2] - lp[2]};
            const double dist = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
            const double rr = grown(p, dm);
            LbJob::Cone c;
            for (int k = 0; k < 3; k++) c.u[k] = dist > 0 ? w[k] / dist : (k == 0 ? 1.0 : 0.0);
            if (dist - rr >= LB_RHO) {
                c.alpha = std::asin(std::min(1.0, rr / dist)) + LB_MU * (double)(1 << t);
            } else {  // (lb_near_all tiers only) within LB_RHO of the light: every cell
                c.alpha = PI;
            }
            c.ca = std::cos(c.alpha);
            c.sa = std::sin(c.alpha);
            c.near = std::max(0.0, dist - rr);
            c.code = p.code;
            c.prev_same = -1;
            c.faces = 0;
            c.all = false;
            for (int f = 0; f < 6; f++) {  // the angle to the face's axis
                const int k = f >> 1;
                const double sg = (f & 1) ? -1.0 : 1.0;
                const double ax_ang = std::acos(std::max(-1.0, std::min(1.0, sg * c.u[k])));
                if (!(ax_ang > c.alpha + FACE_HALF + 1e-3)) c.faces |= (uint8_t)(1u << f);
            }
            cones.push_back(c);
        }
        // nearest first: every cell's list comes out sorted by distance from the light
        std::stable_sort(cones.begin(), cones.end(),
                         [](const LbJob::Cone& a, const LbJob::Cone& b) { return a.near < b.near; });
        std::vector<std::pair<uint32_t, int>> byc(cones.size());
        for (size_t i = 0; i < cones.size(); i++) byc[i] = std::make_pair(cones[i].code, (int)i);
        std::sort(byc.begin(), byc.end());
        for (size_t i = 1; i < byc.size(); i++)
            if (byc[i].first == byc[i - 1].first) cones[byc[i].second].prev_same = byc[i - 1].second;
        // records with a cone over every direction: into the all-cell leaf (every cone of the
        // record leaves the cell lists), nearest first, at the record's nearest distance
        for (size_t lo = 0, hi; lo < byc.size(); lo = hi) {
            bool all = false;
            for (hi = lo; hi < byc.size() && byc[hi].first == byc[lo].first; hi++) all = all || cones[byc[hi].second].alpha >= PI;
            if (all)
                for (size_t i = lo; i < hi; i++) cones[byc[i].second].all = true;
        }
        for (const LbJob::Cone& c : cones)  // nearest first: a record's first cone is its nearest
            if (c.all && c.prev_same < 0) jb.all_ent.push_back(LbJob::Ent{c.code, reach_cut ? down_f(c.near) : 0.f});
    });
    // (2) per job and chunk of cones: the (cell, entry) pairs in cone order
    const int CONE_CHUNK = 64;
    std::vector<std::pair<int, int>> units;
    for (size_t ji = 0; ji < jobs.size(); ji++) {
        const int n_chunks = (int)((jobs[ji].cones.size() + CONE_CHUNK - 1) / CONE_CHUNK);
        jobs[ji].chunk_hits.resize(n_chunks);
        for (int c = 0; c < n_chunks; c++) units.push_back(std::make_pair((int)ji, c));
    }
    parallel_jobs((int)units.size(), threads, [&](int ui) {
        LbJob& jb = jobs[units[ui].first];
        const std::vector<LbJob::Cone>& cones = jb.cones;
        auto cell_in = [&](const LbJob::Cone& c, int cc) {
            if (c.alpha + crad[cc] >= PI) return true;
            // angle(u, cell centre) <= alpha + cell radius  <=>  dot >= cos(alpha + rad)
            const double dt = c.u[0] * cdir[3 * cc] + c.u[1] * cdir[3 * cc + 1] + c.u[2] * cdir[3 * cc + 2];
            return dt >= c.ca * ccos[cc] - c.sa * csin[cc] - 1e-12;
        };
        auto& hits = jb.chunk_hits[units[ui].second];
        const size_t c0 = (size_t)units[ui].second * CONE_CHUNK, c1 = std::min(cones.size(), c0 + CONE_CHUNK);
        for (size_t ci = c0; ci < c1; ci++) {
            const LbJob::Cone& c = cones[ci];
            if (c.all) continue;  // listed once, in the all-cell leaf
            const LbJob::Ent en{c.code, reach_cut ? down_f(c.near) : 0.f};
            for (int f = 0; f < 6; f++) {
                if (!(c.faces >> f & 1)) continue;
                for (int b = f * NB * NB; b < (f + 1) * NB * NB; b++) {
                    if (c.alpha + brad[b] + 1e-4 < PI) {
                        const double dt = c.u[0] * bdir[3 * b] + c.u[1] * bdir[3 * b + 1] + c.u[2] * bdir[3 * b + 2];
                        if (std::acos(std::max(-1.0, std::min(1.0, dt))) > c.alpha + brad[b] + 1e-4) continue;
                    }
                    const int bj = (b - f * NB * NB) / NB, bi = (b - f * NB * NB) % NB;
                    for (int j = bj * BS; j < std::min(R, bj * BS + BS); j++)
                        for (int i = bi * BS; i < std::min(R, bi * BS + BS); i++) {
                            const int cc = (f * R + j) * R + i;
                            if (!cell_in(c, cc)) continue;
                            // a pair record's partner listed here already: keep the first entry
                            bool dup = false;
                            for (int q = c.prev_same; q >= 0 && !dup; q = cones[q].prev_same)
                                dup = (cones[q].faces >> f & 1) && cell_in(cones[q], cc);
                            if (!dup) hits.push_back(std::make_pair((uint32_t)cc, en));
                        }
                }
            }
        }
    });
    // (3) per job: the entries grouped by cell (stable: nearest first), per cell and type the
    // first copy
    parallel_jobs((int)jobs.size(), threads, [&](int ji) {
        LbJob& jb = jobs[ji];
        jb.cell_start.assign((size_t)nc + 1, 0);
        size_t n = 0;
        for (const auto& hits : jb.chunk_hits) {
            n += hits.size();
            for (const auto& h : hits) jb.cell_start[h.first + 1]++;
        }
        for (int cc = 0; cc < nc; cc++) jb.cell_start[cc + 1] += jb.cell_start[cc];
        jb.ent.resize(n);
        std::vector<uint32_t> fill(jb.cell_start.begin(), jb.cell_start.end() - 1);
        for (auto& hits : jb.chunk_hits) {
            for (const auto& h : hits) jb.ent[fill[h.first]++] = h.second;
            std::vector<std::pair<uint32_t, LbJob::Ent>>().swap(hits);
        }
        jb.cell_first.resize(4 * (size_t)nc);
        for (int cc = 0; cc < nc; cc++) {
            for (int k = 0; k < 4; k++) jb.cell_first[4 * cc + k] = (uint32_t)jb.count[k];
            for (uint32_t e = jb.cell_start[cc]; e < jb.cell_start[cc + 1]; e++) jb.count[jb.ent[e].code >> 30]++;
        }
        for (int k = 0; k < 4; k++) jb.all_first[k] = jb.count[k];
        for (const LbJob::Ent& e : jb.all_ent) jb.count[e.code >> 30]++;
    });
    // the copies' places: each job's copies follow the previous job's, per run array, after
    // the array's own records
    const size_t spare[4] = {15, 15, 20, 15};  // the record slot that carries the nearest distance
    const std::vector<float>* run[4] = {&L.dsph, &L.gsph, &L.tri, &L.cube};
    size_t n_src[4], n_rec[4];
    for (int k = 0; k < 4; k++) n_src[k] = n_rec[k] = run[k]->size() / RUN_WIDTH[k];
    for (LbJob& jb : jobs)
        for (int k = 0; k < 4; k++) {
            jb.first[k] = n_rec[k];
            n_rec[k] += jb.count[k];
        }
    for (int k = 0; k < 4; k++) {
        L.ext[k].lb_floats = (n_rec[k] - n_src[k]) * RUN_WIDTH[k];
        L.ext[k].lb.reset(new float[std::max<size_t>(1, L.ext[k].lb_floats)]);
    }
    L.leaves.resize((size_t)next_leaf * 8);
    // per cell, per type nearest first; each copy carries its nearest distance to the light
    // (down-rounded) in the record's spare slot: the device stops a run at the first record
    // no undecided lane can reach
    const int CELL_CHUNK = 512;
    const int n_cell_chunks = (nc + CELL_CHUNK - 1) / CELL_CHUNK;
    // a leaf's runs, copies at first[k] on (each entry's record, its nearest distance in the spare slot)
    auto emit = [&](uint32_t* leaf, const LbJob::Ent* e0, const LbJob::Ent* e1, const size_t first[4]) {
        for (int k = 0; k < 4; k++) {
            const size_t w = RUN_WIDTH[k];
            size_t at = first[k];
            leaf[2 * k] = (uint32_t)at;
            const float* src = run[k]->data();
            float* dst = L.ext[k].lb.get() - n_src[k] * w;  // record index -> its place
            for (const LbJob::Ent* e = e0; e < e1; e++) {
                if ((int)(e->code >> 30) != k) continue;
                const size_t r = e->code & 0x3FFFFFFFu;  // a hierarchy record (< n_src)
                std::memcpy(dst + w * at, src + w * r, w * sizeof(float));
                dst[w * at + spare[k]] = e->near;
                at++;
            }
            leaf[2 * k + 1] = (uint32_t)at;
        }
    };
    parallel_jobs((int)jobs.size() * n_cell_chunks, threads, [&](int ui) {
        const int ji = ui / n_cell_chunks, c0 = (ui % n_cell_chunks) * CELL_CHUNK, c1 = std::min(nc, c0 + CELL_CHUNK);
        const LbJob& jb = jobs[ji];
        uint32_t* leaf = L.leaves.data() + ((size_t)jb.cell_leaf + c0) * 8;
        for (int cc = c0; cc < c1; cc++, leaf += 8) {
            size_t first[4];
            for (int k = 0; k < 4; k++) first[k] = jb.first[k] + jb.cell_first[4 * cc + k];
            emit(leaf, jb.ent.data() + jb.cell_start[cc], jb.ent.data() + jb.cell_start[cc + 1], first);
            // bit 31 of the first run's start: the tier's all-cell leaf has records (rt_scan.hpp lb_leaf)
            if (!jb.all_ent.empty()) leaf[0] |= 0x80000000u;
        }
        if (c0 == 0) {
            size_t first[4];
            for (int k = 0; k < 4; k++) first[k] = jb.first[k] + jb.all_first[k];
            emit(L.leaves.data() + (size_t)jb.all_leaf * 8, jb.all_ent.data(), jb.all_ent.data() + jb.all_ent.size(), first);
        }
    });
}

// Shape buffers (rt_scan.hpp scan_buffered, key mode 7).  A ray inside a sphere S tests S
// first; its exit t bounds the walk.  If the ray's segment [o, o + t d] lies in S's bounding
// ball B(c, Rc) (the device checks both ends: the ball is convex), every hit nearer than the
// exit lies on that segment, and a hierarchy primitive Q can only report such a hit if the
// point lies within h(D) of Q (the hierarchy's own bound, D <= 3 R inside the scene ball;
// grazing triangles: the grazing pass, which always runs) -- i.e. only if Q's ball, grown by
// h(3 R), meets B(c, Rlist).  Rlist = Rc + 2e-5 (|c| + Rc) covers the f32 rounding of the
// device's check (the ends' distances, o + t d, c); Rc is the ball's radius + 0.1 % (the
// exit point lies on the surface, up to rounding).  S's buffer is a leaf record whose runs
// are copies of the records of every such Q (S itself included); a lane whose check passes
// tests it instead of walking the hierarchy.  Spheres whose list would exceed 96 records
// get no buffer.
void build_shape_buffers(RunLayout& L, std::vector<ShapeRec>& shapes, const Tune& T) {
    if (!T.shape_buf || !L.use || L.lb_prims.empty()) return;
    const double dmax = 3.0 * (double)L.r;
    const double hmax = ((double)L.g2 * dmax + (double)L.g1) * dmax + (double)L.g0;
    for (const LbPrim& P : L.lb_prims) {
        const uint32_t type = P.code >> 30;
        if (type != LB_DSPH && type != LB_GSPH) continue;
        ShapeRec& R = shapes[P.shape];
        if (R.kind != RT_SHAPE_SPHERE || R.pad1 != 0) continue;
        const double cn = std::sqrt(P.c[0] * P.c[0] + P.c[1] * P.c[1] + P.c[2] * P.c[2]);
        // 0.1 % over the ball: the exit point lies on the surface, up to rounding
        const float rc = up_f(P.r * 1.001);
        const double rlist = (double)rc + 2e-5 * (cn + (double)rc);
        std::vector<uint32_t> by[4];
        size_t n_rec = 0;
        for (const LbPrim& Q : L.lb_prims) {
            const double dx = Q.c[0] - P.c[0], dy = Q.c[1] - P.c[1], dz = Q.c[2] - P.c[2];
            if (!(std::sqrt(dx * dx + dy * dy + dz * dz) <= (Q.r + rlist + std::min(Q.h3, hmax)) * (1 + 1e-9))) continue;
            auto& v = by[Q.code >> 30];
            const uint32_t rec = Q.code & 0x3FFFFFFFu;
            if (std::find(v.begin(), v.end(), rec) == v.end()) {
                v.push_back(rec);
                n_rec++;
            }
        }
#if RT_DIAG
        if (std::getenv("RT_DEBUG_SHAPE_BUF"))
            std::fprintf(stderr, "shape %u r %.4f rc %.4f hmax %.5f records %zu\n", P.shape, P.r, (double)rc, hmax, n_rec);
#endif
        if (n_rec == 0 || n_rec > 96) continue;
        uint32_t rec[8];
        // copies of hierarchy records, after the run array's records and light-buffer copies
        const std::vector<float>* runs[4] = {&L.dsph, &L.gsph, &L.tri, &L.cube};
        for (int k = 0; k < 4; k++) {
            const size_t w = RUN_WIDTH[k];
            std::vector<float>& sb = L.ext[k].sb;
            rec[2 * k] = (uint32_t)((runs[k]->size() + L.ext[k].lb_floats + sb.size()) / w);
            for (uint32_t r : by[k]) sb.insert(sb.end(), runs[k]->begin() + w * r, runs[k]->begin() + w * (r + 1));
            rec[2 * k + 1] = (uint32_t)((runs[k]->size() + L.ext[k].lb_floats + sb.size()) / w);
        }
        const uint32_t leaf = (uint32_t)(L.leaves.size() / 8);
        L.leaves.insert(L.leaves.end(), rec, rec + 8);
        R.pad1 = (int32_t)(leaf + 1);
        R.a[0] = (float)P.c[0];
        R.a[1] = (float)P.c[1];
        R.a[2] = (float)P.c[2];
        R.a[3] = rc;
    }
}

void build_runs(const std::vector<SphIn>& sph, const std::vector<TriIn>& tris, const std::vector<CubeIn>& cubes,
                const Tune& tn, RunLayout& L) {
    const bool enable = tn.bvh != 0;
    using namespace rtbvh;
    std::vector<Prim> prims;
    std::vector<Geo> geo;
    std::vector<char> in_sph(sph.size(), 0), in_tri(tris.size(), 0), in_cube(cubes.size(), 0);
    std::vector<double> tri_gsin(tris.size(), 0.0);
    std::vector<double> cube_lf(cubes.size(), 0), cube_sn(cubes.size(), 0);
    // per-primitive bounds as polynomials in D (see rt_scan.hpp): box inflation
    // h = a2 D^2 + a1 D + a0 + cC |C|, t-margin m = b1 D + b0 + bC |C|
    struct Coef {
        double a2, a1, a0, cC, b1, b0, bC;
    };
    std::vector<Coef> coef;
    if (enable) {
        for (size_t i = 0; i < sph.size(); i++) {
            Geo g;
            double sigL, sn, sigA;
            if (!geo_affine(sph[i].inv, false, g, sigL, sn, sigA)) continue;
            // basis r_P (7.5 eps (|l|^2 + 1) + eps (|l| + 1 + |L||o| + |s|)), |l| <= sigma(L) D
            double rP = sigA, S = SAFETY_SPHERE;
            coef.push_back(Coef{S * 7.5 * FEPS * rP * sigL * sigL, S * rP * FEPS * 2.0 * sigL,
                                S * rP * FEPS * (8.5 + sn), S * rP * FEPS * sigL, 0, 0, 0});
            in_sph[i] = 1;
            Prim p;
            p.kind = sph[i].diag ? P_DSPH : P_GSPH;
            p.id = (uint32_t)i;
            std::memcpy(p.lo, g.lo, sizeof(p.lo));
            std::memcpy(p.hi, g.hi, sizeof(p.hi));
            p.cost = sph[i].diag ? 30.0 : 60.0;
            prims.push_back(p);
            geo.push_back(g);
        }
        const bool tris_in_bvh = tn.bvh_tris != 0;  // 0: loose triangles stay linear (A/B)
        for (size_t i = 0; i < tris.size() && tris_in_bvh; i++) {
            const TriIn& t = tris[i];
            double v[3][3] = {{t.v[0].x, t.v[0].y, t.v[0].z}, {t.v[1].x, t.v[1].y, t.v[1].z},
                              {t.v[2].x, t.v[2].y, t.v[2].z}};
            double e1[3], e2[3];
            for (int k = 0; k < 3; k++) {
                e1[k] = v[1][k] - v[0][k];
                e2[k] = v[2][k] - v[0][k];
            }
            double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                           e1[0] * e2[1] - e1[1] * e2[0]};
            double ln = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            double l1 = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
            double l2 = std::sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
            double sin_a = ln / (l1 * l2);
            if (!(sin_a >= MIN_SIN_ALPHA) || !std::isfinite(sin_a)) continue;
            Geo g;
            double rad = 0;
            for (int k = 0; k < 3; k++) {
                g.lo[k] = std::min(v[0][k], std::min(v[1][k], v[2][k]));
                g.hi[k] = std::max(v[0][k], std::max(v[1][k], v[2][k]));
                g.c[k] = (v[0][k] + v[1][k] + v[2][k]) / 3.0;
            }
            for (int j = 0; j < 3; j++) {
                double dx = v[j][0] - g.c[0], dy = v[j][1] - g.c[1], dz = v[j][2] - g.c[2];
                rad = std::max(rad, std::sqrt(dx * dx + dy * dy + dz * dz));
            }
            g.r = rad * (1 + 1e-9);
            // basis eps (|o - v0| + |e|max + |o| + |v0|) / sin(alpha): lateral; the same
            // over sin(phi_min) along the ray (t-margin)
            // the reported hit point lies within rho eps (...) / (sin(alpha) sin(phi)) of the
            // triangle and on the ray, so for sin(phi) >= sin(phi_T) the box grown by that
            // bound contains it: no t-margin needed
            double gs = graze_sin(sin_a, tn.graze_k);
            double k = SAFETY_TRI * FEPS / sin_a * std::max(1.0 / gs, TRI_STEEP);
            double v0n = std::sqrt(v[0][0] * v[0][0] + v[0][1] * v[0][1] + v[0][2] * v[0][2]);
            double e = std::max(l1, l2) + v0n;
            coef.push_back(Coef{0.0, 2.0 * k, k * e, k, 0.0, 0.0, 0.0});
            in_tri[i] = 1;
            tri_gsin[i] = gs;
            Prim p;
            p.kind = P_TRI;
            p.id = (uint32_t)i;
            std::memcpy(p.lo, g.lo, sizeof(p.lo));
            std::memcpy(p.hi, g.hi, sizeof(p.hi));
            p.cost = 26.0;
            prims.push_back(p);
            geo.push_back(g);
        }
        for (size_t i = 0; i < cubes.size(); i++) {
            Geo g;
            double sigL, sn, sigA;
            if (!geo_affine(cubes[i].inv, true, g, sigL, sn, sigA)) continue;
            double S = SAFETY_CUBE;
            // basis sigma(A) eps (|l| + 1 + |L||o| + |s|)
            coef.push_back(Coef{0.0, S * sigA * FEPS * 2.0 * sigL, S * sigA * FEPS * (1.0 + sn),
                                S * sigA * FEPS * sigL, 0, 0, 0});
            cube_lf[i] = sigL;
            cube_sn[i] = sn;
            in_cube[i] = 1;
            Prim p;
            p.kind = P_CUBE;
            p.id = (uint32_t)i;
            std::memcpy(p.lo, g.lo, sizeof(p.lo));
            std::memcpy(p.hi, g.hi, sizeof(p.hi));
            p.cost = 300.0;
            prims.push_back(p);
            geo.push_back(g);
        }
    }
    Tree T = build(prims, tn.bvh_cnode, (size_t)tn.bvh_maxleaf);
    L.use = !prims.empty();
    if (L.use) {
        // scene ball (C, R) around every hierarchy primitive's ball
        for (int k = 0; k < 3; k++) L.c[k] = (float)(0.5 * (T.lo[k] + T.hi[k]));
        double C[3] = {L.c[0], L.c[1], L.c[2]};
        double Cn = std::sqrt(C[0] * C[0] + C[1] * C[1] + C[2] * C[2]);
        double R = 0;
        for (const Geo& g : geo) {
            double dx = g.c[0] - C[0], dy = g.c[1] - C[1], dz = g.c[2] - C[2];
            R = std::max(R, std::sqrt(dx * dx + dy * dy + dz * dz) + g.r);
        }
        R *= 1 + 1e-6;
        double g2 = 0, g1 = 0, g0 = 0, m1 = 0, m0 = 0;
#if RT_DIAG
        if (const char* ss = std::getenv("RT_DEBUG_SPH_SCALE")) {  // measurement only: NOT conservative
            const double k = std::atof(ss);
            for (size_t i = 0; i < coef.size(); i++)
                if (prims[i].kind == P_DSPH || prims[i].kind == P_GSPH) {
                    coef[i].a2 *= k;
                    coef[i].a1 *= k;
                    coef[i].a0 *= k;
                    coef[i].cC *= k;
                }
        }
        if (const char* ts = std::getenv("RT_DEBUG_TRI_SCALE")) {  // measurement only: NOT conservative
            const double k = std::atof(ts);
            for (size_t i = 0; i < coef.size(); i++)
                if (prims[i].kind == P_TRI) {
                    coef[i].a1 *= k;
                    coef[i].a0 *= k;
                    coef[i].cC *= k;
                }
        }
#endif
        for (const Coef& c : coef) {
            g2 = std::max(g2, c.a2);
            g1 = std::max(g1, c.a1);
            g0 = std::max(g0, c.a0 + c.cC * Cn);
            m1 = std::max(m1, c.b1);
            m0 = std::max(m0, c.b0 + c.bC * Cn);
        }
        L.m1 = up_f(m1 * (1 + 1e-6));
        L.m0 = up_f(m0 * (1 + 1e-6));
        g1 += SAFETY_SLAB * 16.0 * FEPS;
        g0 += SAFETY_SLAB * 8.0 * FEPS * (3.0 * Cn + R);
#if RT_DIAG
        if (const char* hs = std::getenv("RT_DEBUG_H_SCALE")) {  // measurement only: NOT conservative
            double k = std::atof(hs);
            g2 *= k;
            g1 *= k;
            g0 *= k;
            m1 *= k;
            m0 *= k;
            L.m1 = up_f(m1);
            L.m0 = up_f(m0);
        }
#endif
        L.r = up_f(R);
        L.g2 = up_f(g2 * (1 + 1e-6));
        L.g1 = up_f(g1 * (1 + 1e-6));
        L.g0 = up_f(g0 * (1 + 1e-6));
        L.root = T.root;
        for (const Node& n : T.nodes) {
            put4(L.nodes, down_f(n.lo[0][0]), down_f(n.lo[1][0]), down_f(n.lo[0][1]), down_f(n.lo[1][1]));
            put4(L.nodes, down_f(n.lo[0][2]), down_f(n.lo[1][2]), up_f(n.hi[0][0]), up_f(n.hi[1][0]));
            put4(L.nodes, up_f(n.hi[0][1]), up_f(n.hi[1][1]), up_f(n.hi[0][2]), up_f(n.hi[1][2]));
            put4(L.nodes, keyf(n.child[0]), keyf(n.child[1]), keyf(n.axis), 0.f);
        }
        auto lb_add = [&](uint32_t pi, uint32_t type, size_t rec) {
            const Geo& g = geo[pi];
            const Prim& p = prims[pi];
            float key = p.kind == P_TRI ? tris[p.id].key : (p.kind == P_CUBE ? cubes[p.id].key : sph[p.id].key);
            uint32_t kb;
            std::memcpy(&kb, &key, 4);
            // the primitive's own polynomial (the hierarchy grows boxes by the maximum over
            // every primitive, which the smallest sphere sets), at D = 3 R, plus the slab terms
            const Coef& q = coef[pi];
            const double d3 = 3.0 * (double)L.r;  // the buffers' D_max
            const double p2 = q.a2, p1 = q.a1 + SAFETY_SLAB * 16.0 * FEPS,
                         p0 = q.a0 + q.cC * Cn + SAFETY_SLAB * 8.0 * FEPS * (3.0 * Cn + R);
            const double h3 = ((p2 * d3 + p1) * d3 + p0) * (1 + 1e-6);
            L.lb_prims.push_back(LbPrim{{g.c[0], g.c[1], g.c[2]}, g.r, (type << 30) | (uint32_t)rec, kb >> 4, h3, p2, p1, p0});
        };
        for (const auto& leaf : T.leaves) {
            std::vector<const SphIn*> ds, gs;
            std::vector<const TriIn*> ts;
            std::vector<uint32_t> cs;
            std::vector<uint32_t> dsi, gsi, tsi, csi;  // their prim indices
            for (uint32_t pi : leaf) {
                const Prim& p = prims[pi];
                if (p.kind == P_DSPH) {
                    ds.push_back(&sph[p.id]);
                    dsi.push_back(pi);
                } else if (p.kind == P_GSPH) {
                    gs.push_back(&sph[p.id]);
                    gsi.push_back(pi);
                } else if (p.kind == P_TRI) {
                    ts.push_back(&tris[p.id]);
                    tsi.push_back(pi);
                } else {
                    cs.push_back(p.id);
                    csi.push_back(pi);
                }
            }
            for (size_t k = 0; k < dsi.size(); k++) lb_add(dsi[k], LB_DSPH, L.dsph.size() / 16 + k / 2);
            for (size_t k = 0; k < gsi.size(); k++) lb_add(gsi[k], LB_GSPH, L.gsph.size() / 16 + k);
            for (size_t k = 0; k < tsi.size(); k++) lb_add(tsi[k], LB_TRI, L.tri.size() / 24 + k / 2);
            for (size_t k = 0; k < csi.size(); k++) lb_add(csi[k], LB_CUBE, L.cube.size() / 16 + k);
            if (ds.size() & 1) ds.push_back(ds.back());  // testing a sphere twice changes nothing
            uint32_t rec[8];
            rec[0] = (uint32_t)(L.dsph.size() / 16);
            for (size_t k = 0; k < ds.size(); k += 2) emit_dsph_pair(L.dsph, *ds[k], *ds[k + 1]);
            rec[1] = (uint32_t)(L.dsph.size() / 16);
            rec[2] = (uint32_t)(L.gsph.size() / 16);
            for (const SphIn* q : gs) emit_gsph(L.gsph, *q);
            rec[3] = (uint32_t)(L.gsph.size() / 16);
            rec[4] = (uint32_t)(L.tri.size() / 24);
            for (size_t k = 0; k < ts.size(); k += 2) {
                const TriIn* b = (k + 1 < ts.size()) ? ts[k + 1] : nullptr;
                emit_tri_pair(L.tri, *ts[k], b);
            }
            rec[5] = (uint32_t)(L.tri.size() / 24);
            rec[6] = (uint32_t)(L.cube.size() / 16);
            for (uint32_t ci : cs) emit_cube(L.cube, cubes[ci], (float)cube_lf[ci], up_f(cube_sn[ci]));
            rec[7] = (uint32_t)(L.cube.size() / 16);
            L.leaves.insert(L.leaves.end(), rec, rec + 8);
        }
#if RT_DIAG
        if (std::getenv("RT_BVH_DEBUG")) {
            size_t kinds[4] = {0, 0, 0, 0}, max_leaf = 0;
            for (const Prim& p : prims) kinds[p.kind]++;
            for (const auto& lf : T.leaves) max_leaf = std::max(max_leaf, lf.size());
            std::fprintf(stderr,
                         "rt_bvh: prims dsph %zu gsph %zu tri %zu cube %zu (of sph %zu tri %zu cube %zu); "
                         "nodes %zu leaves %zu depth %d max_leaf %zu; C (%g %g %g) R %g; h = (%g D + %g) D + %g; "
                         "m = %g D + %g\n",
                         kinds[0], kinds[1], kinds[2], kinds[3], sph.size(), tris.size(), cubes.size(),
                         T.nodes.size(), T.leaves.size(), T.depth, max_leaf, L.c[0], L.c[1], L.c[2], L.r, L.g2,
                         L.g1, L.g0, L.m1, L.m0);
        }
#endif
        build_graze(tris, in_tri, tri_gsin, L, tn);
        L.n_dsph_bvh = (int)(L.dsph.size() / 16);
        L.n_gsph_bvh = (int)(L.gsph.size() / 16);
        L.n_tri_bvh = (int)(L.tri.size() / 24);
        L.n_cube_bvh = (int)(L.cube.size() / 16);
    }
    // ---- the linear rest
    std::vector<const SphIn*> ds;
    for (size_t i = 0; i < sph.size(); i++) {
        if (in_sph[i]) continue;
        if (sph[i].diag) ds.push_back(&sph[i]);
        else emit_gsph(L.gsph, sph[i]);
    }
    for (size_t k = 0; k + 1 < ds.size(); k += 2) emit_dsph_pair(L.dsph, *ds[k], *ds[k + 1]);
    if (ds.size() & 1) emit_gsph(L.gsph, *ds.back());
    std::vector<const TriIn*> ts;
    for (size_t i = 0; i < tris.size(); i++)
        if (!in_tri[i]) ts.push_back(&tris[i]);
    for (size_t k = 0; k < ts.size(); k += 2) emit_tri_pair(L.tri, *ts[k], (k + 1 < ts.size()) ? ts[k + 1] : nullptr);
    for (size_t i = 0; i < cubes.size(); i++)
        if (!in_cube[i]) emit_cube(L.cube, cubes[i], 0.f, 0.f);
}

}  // namespace

namespace rthost {

// The host half of rt_scene_create: every array of the device scene, built from the
// description without a HIP call (rt_scene_layout_digest runs it alone), and the section
// table of the one device allocation.
struct HostScene {
    static constexpr int N_SECS = 16;
    struct Sec {  // a section of the device allocation: up to three host pieces, back to back
        const void* src[3];
        size_t bytes[3];
        size_t off;
        size_t size() const { return bytes[0] + bytes[1] + bytes[2]; }
    };
    std::vector<float> dsph, gsph, tri, cube, plane, cubetri;
    std::vector<ShapeRec> shapes;
    std::vector<MatRec> mats;
    std::vector<LightRec> lights;
    RunLayout lay;
    LightBuffers lbuf;
    uint64_t flops = 0;
    uint32_t n_point = 0;
    bool normals_ok = true;
    double nmax = 1.0;
    int n_dsph_all = 0, n_gsph_all = 0, n_tri_all = 0, n_cube_all = 0;
    Sec secs[N_SECS];
    size_t total = 0;
};

namespace {

rt_status prepare_scene(const rt_scene_desc* d, const Tune& tn, HostScene& H) {
    if ((d->n_materials && !d->materials) || (d->n_shapes && !d->shapes) || (d->n_lights && !d->lights))
        return RT_ERR_INVALID_ARG;
    if (d->n_shapes >= (1u << 27)) return RT_ERR_UNSUPPORTED;
    if (d->n_materials > RT_MAX_MATERIALS) return RT_ERR_UNSUPPORTED;  // node_flags holds the index

    // ---- host preprocessing: per-shape records
    std::vector<ShapeRec>& shapes = H.shapes;
    shapes.resize(d->n_shapes);
    std::vector<SphIn> sph_in;
    std::vector<TriIn> tri_in;
    std::vector<CubeIn> cube_in;
    uint64_t& flops = H.flops;
    bool& normals_ok = H.normals_ok;  // DevScene::dark_skip: every hit normal finite with |n| <= 1e3
    double& nmax = H.nmax;    // largest hit-normal length (unit normals; planes: |transform * n|)
    for (uint32_t i = 0; i < d->n_shapes; i++) {
        const rt_shape& s = d->shapes[i];
        if (s.material < 0 || (uint32_t)s.material >= d->n_materials) return RT_ERR_BAD_MATERIAL;
        ShapeRec& R = shapes[i];
        std::memset(&R, 0, sizeof(R));
        R.kind = s.kind;
        R.mat = s.material;
        M4 inv;
        if (!gj_inverse(s.transform, inv)) return RT_ERR_SINGULAR_MATRIX;  // set_transform
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 4; c++) {
                R.inv[r * 4 + c] = inv.m[r][c];
                if (!(std::fabs(inv.m[r][c]) < 1e18f)) normals_ok = false;  // sphere / cube normals
            }
        float key = keyf(i << 4);
        switch (s.kind) {
            case RT_SHAPE_SPHERE: {
                SphIn q;
                std::memcpy(q.inv, R.inv, sizeof(q.inv));
                q.key = key;
                q.diag = inv.m[0][1] == 0.f && inv.m[0][2] == 0.f && inv.m[1][0] == 0.f &&
                         inv.m[1][2] == 0.f && inv.m[2][0] == 0.f && inv.m[2][1] == 0.f;
                sph_in.push_back(q);
                flops += 57;
                break;
            }
            case RT_SHAPE_PLANE: {
                F3 o = f3(s.data[0], s.data[1], s.data[2]);
                F3 n = f3(s.data[3], s.data[4], s.data[5]);
                // Plane::new axes (plane.rs:22-42)
                F3 w = (flen(fcross(n, f3(1.f, 0.f, 0.f))) <= EPS) ? f3(0.f, 1.f, 0.f) : f3(1.f, 0.f, 0.f);
                F3 u = fnorm(fcross(n, w));
                F3 v = fnorm(fcross(n, u));
                F3 tn = vec3_mul(s.transform, n);  // `self.transform * self.normal` (plane.rs:79)
                if (!(std::fabs(tn.x) <= 1e3f && std::fabs(tn.y) <= 1e3f && std::fabs(tn.z) <= 1e3f)) normals_ok = false;
                nmax = std::max(nmax, std::sqrt((double)tn.x * tn.x + (double)tn.y * tn.y + (double)tn.z * tn.z));
                const float a[15] = {n.x, n.y, n.z, o.x, o.y, o.z, tn.x, tn.y, tn.z, u.x, u.y, u.z, v.x, v.y, v.z};
                std::memcpy(R.a, a, sizeof(a));
                for (int r = 0; r < 3; r++) put4(H.plane, inv.m[r][0], inv.m[r][1], inv.m[r][2], inv.m[r][3]);
                put4(H.plane, n.x, n.y, n.z, key);
                put4(H.plane, o.x, o.y, o.z, 0.f);
                flops += 49;
                break;
            }
            case RT_SHAPE_TRIANGLE: {
                TriIn q;
                q.v[0] = f3(s.data[0], s.data[1], s.data[2]);
                q.v[1] = f3(s.data[3], s.data[4], s.data[5]);
                q.v[2] = f3(s.data[6], s.data[7], s.data[8]);
                q.e1 = fsub(q.v[1], q.v[0]);
                q.e2 = fsub(q.v[2], q.v[0]);
                q.key = key;
                F3 nn = tri_normal(q.v[0], q.v[1], q.v[2]);
                if (!(std::isfinite(nn.x) && std::isfinite(nn.y) && std::isfinite(nn.z))) normals_ok = false;
                const float a[12] = {q.v[0].x, q.v[0].y, q.v[0].z, q.e1.x, q.e1.y, q.e1.z,
                                     q.e2.x, q.e2.y, q.e2.z, nn.x, nn.y, nn.z};
                std::memcpy(R.a, a, sizeof(a));
                tri_in.push_back(q);
                flops += 52;
                break;
            }
            case RT_SHAPE_CUBE: {
                CubeIn q;
                std::memcpy(q.inv, R.inv, sizeof(q.inv));
                q.key = key;
                cube_in.push_back(q);
                flops += 33 + 12 * 52;
                break;
            }
            default:
                return RT_ERR_INVALID_ARG;
        }
    }
    if (d->n_lights > RT_MAX_LIGHTS) return RT_ERR_UNSUPPORTED;  // the shadow keys' light index (16 bits)
    std::vector<LightRec>& lights = H.lights;
    lights.resize(d->n_lights);
    for (uint32_t i = 0; i < d->n_lights; i++) {
        const rt_light& l = d->lights[i];
        if (l.kind != RT_LIGHT_POINT && l.kind != RT_LIGHT_AMBIENT) return RT_ERR_INVALID_ARG;
        lights[i] = LightRec{l.kind, l.pos[0], l.pos[1], l.pos[2], l.color.r, l.color.g, l.color.b, 0xFFFFFFFFu};
        if (l.kind == RT_LIGHT_POINT) H.n_point++;
    }
    // ---- culling hierarchy and the run layout (leaf order first, then the linear rest)
    RunLayout& lay = H.lay;
    build_runs(sph_in, tri_in, cube_in, tn, lay);
    // light buffers append cell leaves and record copies to the layout (after the linear
    // rest: the scan's run counts below exclude them)
    H.n_dsph_all = (int)(lay.dsph.size() / 16);
    H.n_gsph_all = (int)(lay.gsph.size() / 16);
    H.n_tri_all = (int)(lay.tri.size() / 24);
    H.n_cube_all = (int)(lay.cube.size() / 16);
    // the Morton code (morton15, rt_wavefront.hip) of every sphere's and cube's centre -- the
    // forward transform's translation: the task key of rays inside the shape
    if (lay.use) {
        const float sc = 16.f / lay.r;
        auto cell = [&](float p, float c) { return (uint32_t)(int)std::fmin(std::fmax((p - c) * sc + 16.f, 0.f), 31.f); };
        auto spread5 = [](uint32_t v) {
            v = (v | (v << 8)) & 0x0300F00Fu;
            v = (v | (v << 4)) & 0x030C30C3u;
            v = (v | (v << 2)) & 0x09249249u;
            return v;
        };
        for (uint32_t i = 0; i < d->n_shapes; i++) {
            const rt_shape& sh = d->shapes[i];
            if (sh.kind != RT_SHAPE_SPHERE && sh.kind != RT_SHAPE_CUBE) continue;
            const uint32_t x = cell(sh.transform[3], lay.c[0]), y = cell(sh.transform[7], lay.c[1]),
                           z = cell(sh.transform[11], lay.c[2]);
            shapes[i].center_key = (spread5(x) << 2) | (spread5(y) << 1) | spread5(z);
        }
    }
    LightBuffers& lbuf = H.lbuf;
    build_light_buffers(lay, lights, lbuf, tn);
    for (size_t i = 0; i < lights.size(); i++) lights[i].lb_base = lbuf.base[i];
    build_shape_buffers(lay, shapes, tn);
    H.dsph.swap(lay.dsph);
    H.gsph.swap(lay.gsph);
    H.tri.swap(lay.tri);
    H.cube.swap(lay.cube);
    cube_triangles(H.cubetri);
    if (!rt_cube_table_check(H.cubetri.data())) return RT_ERR_UNSUPPORTED;
    std::vector<MatRec>& mats = H.mats;
    mats.resize(d->n_materials);
    for (uint32_t i = 0; i < d->n_materials; i++) {
        rt_status r = mat_rec(d->materials[i], mats[i], nmax);
        if (r != RT_OK) return r;
    }
    // ---- one allocation, 256-B aligned sections
    static const unsigned long long zero_ops[RT_OPS_SLOTS * RT_OPS_STRIDE] = {0};
    auto one = [](const void* p, size_t n) { return HostScene::Sec{{p, nullptr, nullptr}, {n, 0, 0}, 0}; };
    // a run array: its records, the light buffers' copies, the shape buffers' copies
    auto run = [&](const std::vector<float>& v, int k) {
        const RunLayout::Ext& e = lay.ext[k];
        return HostScene::Sec{{v.data(), e.lb.get(), e.sb.data()}, {v.size() * 4, e.lb_floats * 4, e.sb.size() * 4}, 0};
    };
    const HostScene::Sec secs[HostScene::N_SECS] = {
        run(H.dsph, LB_DSPH), run(H.gsph, LB_GSPH), run(H.tri, LB_TRI), run(H.cube, LB_CUBE),
        one(H.plane.data(), H.plane.size() * 4), one(H.cubetri.data(), H.cubetri.size() * 4),
        one(shapes.data(), shapes.size() * sizeof(ShapeRec)),
        one(mats.data(), mats.size() * sizeof(MatRec)),
        one(lights.data(), lights.size() * sizeof(LightRec)),
        one(lay.nodes.data(), lay.nodes.size() * 4),
        one(lay.leaves.data(), lay.leaves.size() * 4),
        one(lay.graze_blk.data(), lay.graze_blk.size() * 4),
        one(zero_ops, sizeof(zero_ops)),
        one(lay.graze_tri.data(), lay.graze_tri.size() * 4),
        one(lay.graze_pn.data(), lay.graze_pn.size() * 4),
        one(lay.graze_mask.data(), lay.graze_mask.size() * 4)};
    size_t total = 0;
    for (int k = 0; k < HostScene::N_SECS; k++) {
        H.secs[k] = secs[k];
        H.secs[k].off = total;
        total += (secs[k].size() + 96 + 255) & ~(size_t)255;  // + one record group of look-ahead slack
    }
    H.total = total == 0 ? 256 : total;
    return RT_OK;
}

}  // namespace

void HostSceneDeleter::operator()(HostScene* h) const { delete h; }

rt_status host_scene_build(const rt_scene_desc* d, const Tune& tn, HostScenePtr& out) {
    HostScenePtr H(new (std::nothrow) HostScene());
    if (!H) return RT_ERR_OUT_OF_MEMORY;
    rt_status st = prepare_scene(d, tn, *H);
    if (st != RT_OK) return st;
    out = std::move(H);
    return RT_OK;
}

size_t host_scene_bytes(const HostScene& H) { return H.total; }

void host_scene_pieces(const HostScene& H, std::vector<UploadPiece>& out) {
    out.clear();
    for (const auto& s : H.secs)
        for (size_t p = 0, at = s.off; p < 3; at += s.bytes[p], p++)
            if (s.bytes[p]) out.push_back(UploadPiece{at, s.src[p], s.bytes[p]});
}

void host_scene_bind(const HostScene& H, const void* dmem, const rt_scene_desc* d, const Tune& tn, DevScene& S,
                     SceneFacts& facts) {
    auto at = [&](int k) { return (const void*)((const uint8_t*)dmem + H.secs[k].off); };
    S.dsph = (const float4*)at(0);
    S.gsph = (const float4*)at(1);
    S.tri = (const float4*)at(2);
    S.cube = (const float4*)at(3);
    S.plane = (const float4*)at(4);
    S.cubetri = (const float4*)at(5);
    S.shapes = (const ShapeRec*)at(6);
    S.mats = (const MatRec*)at(7);
    S.lights = (const LightRec*)at(8);
    S.n_dsph = H.n_dsph_all;  // pairs (light-buffer copies follow)
    S.n_gsph = H.n_gsph_all;
    S.n_tri = H.n_tri_all;    // pairs
    S.n_cube = H.n_cube_all;
    S.n_plane = (int32_t)(H.plane.size() / 20);
    S.n_shapes = (int32_t)d->n_shapes;
    S.n_lights = (int32_t)d->n_lights;
    S.n_mats = (int32_t)d->n_materials;
    S.bvh_nodes = (const float4*)at(9);
    S.bvh_leaves = (const uint4*)at(10);
    S.graze_blk = (const float4*)at(11);
    S.scan_ops = (unsigned long long*)at(12);
    S.graze_tri = (const float4*)at(13);
    S.graze_pn = (const float4*)at(14);
    S.graze_mask = (const uint32_t*)at(15);
    S.graze_res = H.lay.graze_res;
    S.graze_words = H.lay.graze_words;
    S.graze_lane = tn.graze_lane ? 1u : 0u;  // 0: the wave-union grazing path (A/B)
    S.lb_res = H.lbuf.res;
    S.lb_dmax = H.lbuf.dmax;
    S.lb_tiers = H.lbuf.tiers;
    S.n_graze_blk = (int32_t)(H.lay.graze_blk.size() / 32);
#if RT_DIAG
    if (std::getenv("RT_DEBUG_NO_GRAZE")) S.n_graze_blk = 0;  // measurement only: NOT exact (the grazing pass's cost)
#endif
    S.bvh_root = H.lay.root;
    S.n_bvh_nodes = (int32_t)(H.lay.nodes.size() / 16);
    S.use_bvh = H.lay.use ? 1 : 0;
    S.n_dsph_bvh = H.lay.n_dsph_bvh;
    S.n_gsph_bvh = H.lay.n_gsph_bvh;
    S.n_tri_bvh = H.lay.n_tri_bvh;
    S.n_cube_bvh = H.lay.n_cube_bvh;
    S.bvh_cx = H.lay.c[0];
    S.bvh_cy = H.lay.c[1];
    S.bvh_cz = H.lay.c[2];
    S.bvh_r = H.lay.r;
    S.bvh_g2 = H.lay.g2;
    S.bvh_g1 = H.lay.g1;
    S.bvh_g0 = H.lay.g0;
    S.bvh_m1 = H.lay.m1;
    S.bvh_m0 = H.lay.m0;
    S.graze_s2 = 1.0201f;  // normals pre-divided by sin(phi_T): checked at 1.01 sin(phi_T)
#if RT_DIAG
    if (const char* e = std::getenv("RT_DEBUG_GRAZE_S2")) S.graze_s2 = (float)std::atof(e);  // measurement only: NOT exact
#endif
    S.dark_skip = (H.normals_ok && tn.dark_skip) ? 1 : 0;
    S.amb_r = d->ambient.r;
    S.amb_g = d->ambient.g;
    S.amb_b = d->ambient.b;
    facts.flops_per_scan = H.flops;
    facts.n_point_lights = H.n_point;
    facts.normal_max = H.nmax;
}

rt_status material_record(const rt_material& m, MatRec& M, double normal_max) { return mat_rec(m, M, normal_max); }

}  // namespace rthost

using namespace rthost;

extern "C" {

rt_status rt_scene_layout_digest(const rt_scene_desc* d, const char* tuning, uint64_t* digest, uint64_t* bytes) {
    if (!d || !digest) return RT_ERR_INVALID_ARG;
    Tune tn;
    if (!tune_apply(tn, std::getenv("RT_TUNE"), true) || !tune_apply(tn, tuning, true)) return RT_ERR_INVALID_ARG;
    HostScene H;
    rt_status st = prepare_scene(d, tn, H);
    if (st != RT_OK) return st;
    // FNV-1a over the image the device allocation would hold (padding as zeros)
    uint64_t h = 0xcbf29ce484222325ull;
    auto mix = [&](const uint8_t* p, size_t n) {
        for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
    };
    size_t at = 0;
    const uint8_t z[256] = {0};
    for (const auto& s : H.secs) {
        for (; at < s.off; at += std::min<size_t>(256, s.off - at)) mix(z, std::min<size_t>(256, s.off - at));
        for (int p = 0; p < 3; p++) mix((const uint8_t*)s.src[p], s.bytes[p]);
        at += s.size();
    }
    for (; at < H.total; at += std::min<size_t>(256, H.total - at)) mix(z, std::min<size_t>(256, H.total - at));
    const uint64_t tail[4] = {H.flops, H.n_point, (uint64_t)H.normals_ok, (uint64_t)H.lbuf.tiers};
    mix((const uint8_t*)tail, sizeof(tail));
    *digest = h;
    if (bytes) *bytes = H.total;
    return RT_OK;
}

}  // extern "C"
