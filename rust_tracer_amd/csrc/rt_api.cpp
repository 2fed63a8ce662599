// rt_api.cpp -- implementation of the C ABI (include/rt_api.h).
//
// Host side of the boundary: validate the flat scene description, run the scene-build
// preprocessing the reference performs in its constructors and set_transform calls
// (Matrix::inverse matrix.rs:99-153, Plane::new axes plane.rs:22-42, Triangle::new
// normal triangle.rs:16-39, Cube::new triangles cube.rs:21-77), lay the result out as
// the device runs of rt_device.hpp and upload it.  Rendering launches the level-synchronous
// pipeline of rt_wavefront.hip (trace / shadow / combine) with the queue sorts of
// rt_order.hip; there is no CPU fallback anywhere in this library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <atomic>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include <sched.h>

#include "../../include/rt_api.h"
#include "rt_bvh.hpp"
#include "rt_device.hpp"
#include "rt_internal.hpp"
#include "rt_tune.hpp"

namespace rtdev {
hipError_t launch_unpermute(const float* in, uint32_t x_res, uint32_t y_res, uint32_t band_rows,
                            uint32_t world, uint32_t rows_per_rank, float* out, hipStream_t stream,
                            uint32_t frames = 1, uint32_t rank_rows = 0);
hipError_t launch_quantize(const float* in, size_t n, uint8_t* out, hipStream_t stream);
hipError_t launch_unpermute_u8(const uint8_t* in, uint32_t x_res, uint32_t y_res, uint32_t band_rows,
                               uint32_t world, uint32_t rows_per_rank, uint8_t* out, hipStream_t stream,
                               uint32_t frames = 1, uint32_t rank_rows = 0);
bool rt_cube_table_check(const float* table);
hipError_t wave_occupancy(const WaveParams& p, int* trace_blocks, int* shadow_blocks, int* combine_blocks,
                          int* trace_each);
hipError_t launch_wave_shadow(const WaveParams& p, int blocks, hipStream_t stream);
hipError_t launch_wave_init(uint32_t* levels, uint32_t n_words, uint32_t total_items, uint32_t* overflow,
                            hipStream_t stream);
hipError_t launch_wave_trace(const WaveParams& p, uint32_t level, int blocks, hipStream_t stream,
                             const int* occ_each = nullptr, int occ_min = 0);
hipError_t launch_wave_combine(const WaveParams& p, uint32_t level, int blocks, hipStream_t stream);
hipError_t launch_forest_shade(const WaveParams& p, uint32_t level, int blocks, float* frame, hipStream_t stream);
hipError_t launch_forest_mark(const uint32_t* node_key, const uint32_t* node_pixel, const uint32_t* node_flags,
                              uint32_t n_nodes, const uint8_t* key_mask, uint32_t n_keys, uint8_t* mark,
                              uint32_t* sizes, hipStream_t stream);
hipError_t launch_sort(const uint32_t* levels, int32_t level, uint32_t cap, uint32_t bits, const uint32_t* keys,
                       const uint32_t* vals, uint32_t* tmp, uint32_t* vals_out,
                         uint32_t* tile_counts, uint32_t* digit_totals, int blocks, hipStream_t stream,
                         uint32_t max_digit);
uint32_t sort_max_tiles(uint32_t cap);
uint32_t sort_max_digits();
hipError_t launch_spp_accumulate(const float* samples, uint32_t n, size_t frame_floats, uint32_t first, uint32_t spp,
                                 float* out, uint8_t* out8, hipStream_t stream);
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

struct Workspace {
    float* out = nullptr;            // device frame (rt_render)
    size_t out_floats = 0;
    uint8_t* out8 = nullptr;
    size_t out8_bytes = 0;
    unsigned long long* counters = nullptr;  // [node, shadow, pixels, wave iterations]
    uint32_t* work = nullptr;        // persistent-kernel work counter
    // level-synchronous pipeline: the node arrays of rt_device.hpp
    Task* tasks = nullptr;
    uint32_t* node_flags = nullptr;  // [capacity]
    float4* node_ps = nullptr;       // [capacity] shadow-ray origins, texture u
    float4* node_n = nullptr;        // [capacity] normals, texture v
    float4* node_d = nullptr;        // [capacity] ray directions, parents
    uint32_t* node_lit = nullptr;    // [capacity] unshadowed-light bits (lights 0-31)
    uint32_t* node_lit_hi = nullptr; // [(lit_words - 1) x capacity] lights 32 and up
    uint32_t lit_words = 1;          // ceil(lights / 32) (rt_device.hpp WaveParams::lit_words)
    float4* node_ec = nullptr;       // [2 x capacity] children's colours
    uint32_t capacity = 0;
    uint32_t* shadow = nullptr;      // shadow queue
    uint32_t* shadow_light = nullptr;  // wide entries (> 256 lights): each entry's light
    uint32_t shadow_capacity = 0;
    uint32_t* levels = nullptr;      // RT_LEVEL_TABLE_WORDS words
    uint32_t* overflow = nullptr;    // [0] this pass's queue overflows, [1] sticky (rt_scene_sync_status)
    uint64_t* ctr_save = nullptr;    // a checked pass's caller counters before it (rt_render_bands_ex_async)
    // queue ordering (rt_order.hip)
    uint32_t* task_keys = nullptr;   // [capacity] x2 buffers
    uint32_t* perm = nullptr;
    uint32_t sort_capacity = 0;
    uint32_t* shadow_keys = nullptr; // [shadow_capacity] x2 buffers
    uint32_t* shadow_sorted = nullptr;
    uint32_t sort_shadow_capacity = 0;
    uint32_t* sort_tmp = nullptr;    // scratch keys + values, 256 x tiles counts, 256 digit totals
    size_t sort_tmp_words = 0;
    // ray forest only (rt_forest): per-node shade inputs, grown with the pool
    bool forest = false;
    float4* node_dc = nullptr;       // [2 x capacity] children's directions
    uint32_t* node_key = nullptr;
    uint32_t* node_pixel = nullptr;
    // sample batches: one band buffer per sample of a batch (launch_bands_wave)
    float* spp_buf = nullptr;
    size_t spp_buf_floats = 0;
};

// Task ordering key (rt_wavefront.hip task_key / inside_key; Tune::task_key): 7 (default) =
// a ray inside a sphere or cube (the refracted child of an entering hit, the reflected child
// of a hit from inside) is keyed by that shape's centre (1 | 15-bit Morton of the centre), so
// a wave holds the rays trapped in one or two shapes; every other ray by face x 2x2
// direction cells | 10-bit Morton code of a point 0.25 x (scene radius) ahead on the ray
// (mode 6 with one bit less).  Measured alternatives (config 3, 1080p): 1 = face
// x 2x2 cells | 11-bit Morton origin 4.90 ms, 6 at 0.10 - 0.35 ahead 4.81 - 4.94, 5 (0.5
// ahead) +1.5%, 3 / 4 (24-bit keys) 6.13 / 6.42 vs 5.78 for mode 1.

int g_num_cus(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 256;
    return prop.multiProcessorCount;
}

}  // namespace

struct rt_scene {
    int device = 0;
    void* dmem = nullptr;
    size_t dbytes = 0;
    DevScene S;
    uint64_t flops_per_scan = 0;
    uint32_t n_point_lights = 0;
    int num_cus = 256;
    int occ_trace = 0, occ_shadow = 0, occ_combine = 0;
    int occ_trace_each[3] = {0, 0, 0};  // generic / level-0 / deep trace instantiations
    bool count_ops = false;  // rt_scene_set_scan_counting
    int grid_pct = 100;      // rt_scene_set_grid_share: % of a full chip for persistent grids
    Tune tune;               // rt_tune.hpp: fixed scene-build keys, pass keys (rt_scene_set_tuning)
    Workspace ws;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // one event per stream a stream-ordered render ran on, recorded after each such render:
    // rt_scene_sync_status and rt_scene_destroy wait for every one of them
    std::vector<std::pair<hipStream_t, hipEvent_t>> ev_streams;
    uint32_t pool_floor = 0;       // node-pool size the next pass grows to (after a reported overflow)
    double normal_max = 1.0;       // largest hit-normal length (dark_zero of an edited material)
    rt_multi_state* multi = nullptr;  // rt_scene_create_multi: the other devices' clones (rt_multi.cpp)
    rt_multi_state* split = nullptr;  // rt_render's band shares on this one device (seam_split)
    int split_n = 0;
    uint32_t seam_rows = 0, seam_y = 0;  // the two shares' meeting row (adapted per render) for y_res seam_y
    // rt_render_frame_async (on `split`, rt_render's shares): its meeting row for y_res
    // split_dev_y, whether a render awaits rt_scene_sync_status, and an overflow of such a
    // render that rt_render's own status check found first (reported by the next
    // rt_scene_sync_status)
    uint32_t split_dev_rows = 0, split_dev_y = 0;
    bool split_dev_pending = false, split_dev_overflow = false;
    // rt_render_bands_ex_async: the largest pass (level-0 items, depth) checked for overflow on
    // this handle, and an overflow of an earlier pass that such a check found latched
    // (reported by sync_status)
    uint64_t checked_items = 0;
    uint32_t checked_depth = 0;
    bool ovf_pending = false;
    // the description the device scene was built from (rt_scene_update compares against it)
    std::vector<rt_material> d_mats;
    std::vector<rt_shape> d_shapes;
    std::vector<rt_light> d_lights;
    rt_color d_ambient{0.f, 0.f, 0.f};
    // bumped by every rebuild rt_scene_update adopts: a forest made before it refuses to shade
    // (its trees hold the old scene's material indices and light count)
    uint64_t generation = 0;
    // rt_scene_set_kernel_timing: HIP events around every launch of this handle's passes, by
    // kernel kind (RT_KT_*), summed by rt_scene_kernel_times
    bool ktime = false;
    std::vector<hipEvent_t> kt_events;        // pool, reused
    std::vector<std::pair<int, size_t>> kt_spans;  // (kind, index of the start event; end = +1)
    size_t kt_used = 0;
};

namespace {
// Brackets one launch of kind `kind` with a pair of events when the handle times its kernels.
struct KSpan {
    rt_scene* s;
    hipStream_t st;
    size_t at = 0;
    bool on = false;
    KSpan(rt_scene* sc, hipStream_t stream, int kind) : s(sc), st(stream) {
        if (!s->ktime) return;
        if (s->kt_used + 2 > s->kt_events.size()) {
            for (int i = 0; i < 64; i++) {
                hipEvent_t e = nullptr;
                if (hipEventCreate(&e) != hipSuccess) return;
                s->kt_events.push_back(e);
            }
        }
        at = s->kt_used;
        s->kt_used += 2;
        on = hipEventRecord(s->kt_events[at], st) == hipSuccess;
        if (on) s->kt_spans.emplace_back(kind, at);
    }
    ~KSpan() {
        if (on) (void)hipEventRecord(s->kt_events[at + 1], st);
    }
};
}  // namespace

rt_multi_state*& rt_scene_multi(rt_scene* s) { return s->multi; }
int rt_scene_device_of(const rt_scene* s) { return s->device; }
const Tune& rt_scene_tune(const rt_scene* s) { return s->tune; }

namespace {

rt_status hip_status(hipError_t e) {
    if (e == hipSuccess) return RT_OK;
    if (e == hipErrorOutOfMemory) return RT_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return RT_ERR_NO_DEVICE;
    return RT_ERR_HIP;
}
// a failing HIP call is reported on stderr (expression, line, HIP's message)
#define HIP_TRY(x)                                                                                   \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            std::fprintf(stderr, "rt_api.cpp:%d: %s: %s\n", __LINE__, #x, hipGetErrorString(e_));  \
            return hip_status(e_);                                                                   \
        }                                                                                            \
    } while (0)

rt_status select_device(int32_t device, int* resolved) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_ERR_NO_DEVICE;
    int d = device;
    if (d < 0) HIP_TRY(hipGetDevice(&d));
    if (d >= n) return RT_ERR_NO_DEVICE;
    HIP_TRY(hipSetDevice(d));
    *resolved = d;
    return RT_OK;
}

// Shadow entries: packed (node << bits) | light in 4 B for scenes of up to 256 lights (8 bits);
// "wide" above that -- the node in shadow[], its light in shadow_light[] (rt_device.hpp), so that
// a scene of many lights keeps the full node pool (RT_MAX_LIGHTS).
constexpr uint32_t PACKED_LIGHT_BITS = 8;
uint32_t light_index_bits(const rt_scene* s) {
    uint32_t b = 1;
    while ((1u << b) < (uint32_t)s->S.n_lights) b++;
    return b;
}
bool wide_entries(const rt_scene* s) { return light_index_bits(s) > PACKED_LIGHT_BITS; }
uint32_t light_bits(const rt_scene* s) { return wide_entries(s) ? 0u : light_index_bits(s); }
// Largest node pool: node indices must fit a packed shadow entry beside the light index (and
// (node << 1) | slot a parent reference).
uint64_t pool_cap_limit(const rt_scene* s) { return std::min<uint64_t>(1ull << (32 - light_bits(s)), 1ull << 30); }


rt_status ensure_ws(rt_scene* s, size_t out_floats, size_t out8_bytes) {
    Workspace& w = s->ws;
    if (!w.counters) {
        HIP_TRY(hipMalloc(&w.counters, 4 * sizeof(unsigned long long)));
        HIP_TRY(hipMalloc(&w.work, 64));
        HIP_TRY(hipMalloc(&w.ctr_save, 64));
    }
    if (out_floats > w.out_floats) {
        if (w.out) (void)hipFree(w.out);
        w.out = nullptr;
        w.out_floats = 0;
        HIP_TRY(hipMalloc(&w.out, out_floats * sizeof(float)));
        w.out_floats = out_floats;
    }
    if (out8_bytes > w.out8_bytes) {
        if (w.out8) (void)hipFree(w.out8);
        w.out8 = nullptr;
        w.out8_bytes = 0;
        HIP_TRY(hipMalloc(&w.out8, out8_bytes));
        w.out8_bytes = out8_bytes;
    }
    return RT_OK;
}

// (Re)allocates every per-node array with `cap` slots: tasks, the node arrays
// (rt_device.hpp).  The per-node sort buffers follow lazily (sort_capacity < capacity),
// the shadow queue from capacity * point lights.
rt_status grow_node_pool(Workspace& w, uint32_t cap) {
    for (void** b : {(void**)&w.tasks, (void**)&w.node_flags, (void**)&w.node_ps, (void**)&w.node_n,
                     (void**)&w.node_d, (void**)&w.node_lit, (void**)&w.node_lit_hi, (void**)&w.node_ec, (void**)&w.node_dc,
                     (void**)&w.node_key, (void**)&w.node_pixel}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    w.capacity = 0;
    HIP_TRY(hipMalloc(&w.tasks, (size_t)cap * sizeof(Task)));
    HIP_TRY(hipMalloc(&w.node_flags, (size_t)cap * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&w.node_ps, (size_t)cap * sizeof(float4)));
    HIP_TRY(hipMalloc(&w.node_n, (size_t)cap * sizeof(float4)));
    HIP_TRY(hipMalloc(&w.node_d, (size_t)cap * sizeof(float4)));
    HIP_TRY(hipMalloc(&w.node_lit, (size_t)cap * sizeof(uint32_t)));
    if (w.lit_words > 1) HIP_TRY(hipMalloc(&w.node_lit_hi, (size_t)(w.lit_words - 1) * cap * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&w.node_ec, 2 * (size_t)cap * sizeof(float4)));
    if (w.forest) {
        HIP_TRY(hipMalloc(&w.node_dc, 2 * (size_t)cap * sizeof(float4)));
        HIP_TRY(hipMalloc(&w.node_key, (size_t)cap * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&w.node_pixel, (size_t)cap * sizeof(uint32_t)));
    }
    w.capacity = cap;
    return RT_OK;
}

// Frees every device / pinned buffer of a workspace.
void free_workspace(Workspace& w) {
    for (void* b : {(void*)w.out, (void*)w.out8, (void*)w.counters, (void*)w.work, (void*)w.tasks, (void*)w.shadow,
                    (void*)w.shadow_light,
                    (void*)w.node_flags, (void*)w.levels, (void*)w.overflow, (void*)w.node_ps, (void*)w.node_n,
                    (void*)w.node_d, (void*)w.node_lit, (void*)w.node_lit_hi, (void*)w.node_ec, (void*)w.task_keys, (void*)w.perm,
                    (void*)w.shadow_keys, (void*)w.shadow_sorted, (void*)w.sort_tmp, (void*)w.node_dc,
                    (void*)w.node_key, (void*)w.node_pixel, (void*)w.spp_buf, (void*)w.ctr_save})
        if (b) (void)hipFree(b);
    w = Workspace();
}

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

rt_status create_handle(const rt_scene_desc* d, int32_t device, const Tune& tn, rt_scene** out);

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

extern "C" {

int32_t rt_api_version(void) { return RT_API_VERSION; }
uint32_t rt_max_frames(void) { return RT_MAX_FRAMES; }

const char* rt_status_str(rt_status s) {
    switch (s) {
        case RT_OK: return "RT_OK";
        case RT_ERR_INVALID_ARG: return "RT_ERR_INVALID_ARG";
        case RT_ERR_SINGULAR_MATRIX: return "RT_ERR_SINGULAR_MATRIX";
        case RT_ERR_UNSUPPORTED: return "RT_ERR_UNSUPPORTED";
        case RT_ERR_NO_DEVICE: return "RT_ERR_NO_DEVICE";
        case RT_ERR_HIP: return "RT_ERR_HIP";
        case RT_ERR_OUT_OF_MEMORY: return "RT_ERR_OUT_OF_MEMORY";
        case RT_ERR_BAD_MATERIAL: return "RT_ERR_BAD_MATERIAL";
        case RT_ERR_CAPACITY: return "RT_ERR_CAPACITY";
        default: return "RT_ERR_UNKNOWN";
    }
}

uint32_t rt_band_rows_per_rank(uint32_t y_res, uint32_t band_rows, uint32_t world) {
    if (band_rows == 0 || world == 0) return 0;
    uint32_t n_bands = (y_res + band_rows - 1) / band_rows;
    uint32_t per_rank = (n_bands + world - 1) / world;
    return per_rank * band_rows;
}

rt_status rt_scene_create(const rt_scene_desc* d, int32_t device, rt_scene** out) {
    return rt_scene_create_tuned(d, device, nullptr, out);
}

rt_status rt_scene_create_tuned(const rt_scene_desc* d, int32_t device, const char* tuning, rt_scene** out) {
    if (!d || !out) return RT_ERR_INVALID_ARG;
    // the handle's tuning: defaults, the environment's RT_TUNE (A/B harness), then `tuning`
    Tune tn;
    if (!tune_apply(tn, std::getenv("RT_TUNE"), true) || !tune_apply(tn, tuning, true)) return RT_ERR_INVALID_ARG;
    return create_handle(d, device, tn, out);
}

}  // extern "C"

namespace {

rt_status create_handle(const rt_scene_desc* d, int32_t device, const Tune& tn, rt_scene** out) {
    HostScene H;
    rt_status pst = prepare_scene(d, tn, H);
    if (pst != RT_OK) return pst;
    std::unique_ptr<rt_scene> sc(new (std::nothrow) rt_scene());
    if (!sc) return RT_ERR_OUT_OF_MEMORY;
    rt_status st = select_device(device, &sc->device);
    if (st != RT_OK) return st;
    HIP_TRY(hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&sc->ev0));
    HIP_TRY(hipEventCreate(&sc->ev1));
    HIP_TRY(hipMalloc(&sc->dmem, H.total));
    sc->dbytes = H.total;
    // on the scene's own stream, waited for (the host arrays are pageable and go out of
    // scope): the padding zeroed, then each section straight from its array
    HIP_TRY(hipMemsetAsync(sc->dmem, 0, H.total, sc->stream));
    for (const auto& s : H.secs)
        for (size_t p = 0, at = s.off; p < 3; at += s.bytes[p], p++)
            if (s.bytes[p])
                HIP_TRY(hipMemcpyAsync((uint8_t*)sc->dmem + at, s.src[p], s.bytes[p], hipMemcpyHostToDevice, sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    auto at = [&](int k) { return (const void*)((const uint8_t*)sc->dmem + H.secs[k].off); };
    DevScene& S = sc->S;
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
    sc->flops_per_scan = H.flops;
    sc->n_point_lights = H.n_point;
    sc->normal_max = H.nmax;
    sc->num_cus = g_num_cus(sc->device);
    sc->tune = tn;
    sc->d_mats.assign(d->materials, d->materials + d->n_materials);
    sc->d_shapes.assign(d->shapes, d->shapes + d->n_shapes);
    sc->d_lights.assign(d->lights, d->lights + d->n_lights);
    sc->d_ambient = d->ambient;
    *out = sc.release();
    return RT_OK;
}

// rt_scene_update's rebuild, in two steps so that a failure leaves every handle as it was:
// stage_scene_data waits for dst's renders and copies src's device scene into a new
// allocation on dst's device; commit_scene_data then swaps it in (rebased DevScene, the
// description, the light count's workspace consequences).
rt_status stage_scene_data(rt_scene* dst, const rt_scene* src, void** out) {
    *out = nullptr;
    HIP_TRY(hipSetDevice(dst->device));
    HIP_TRY(hipStreamSynchronize(dst->stream));
    for (auto& se : dst->ev_streams) HIP_TRY(hipEventSynchronize(se.second));  // renders on other streams
    void* mem = nullptr;
    HIP_TRY(hipMalloc(&mem, src->dbytes));
    rt_status st = RT_OK;
    if (dst->device == src->device)
        st = hip_status(hipMemcpyAsync(mem, src->dmem, src->dbytes, hipMemcpyDeviceToDevice, dst->stream));
    else
        st = hip_status(hipMemcpyPeerAsync(mem, dst->device, src->dmem, src->device, src->dbytes, dst->stream));
    if (st == RT_OK) st = hip_status(hipStreamSynchronize(dst->stream));
    if (st != RT_OK) {
        (void)hipFree(mem);
        return st;
    }
    *out = mem;
    return RT_OK;
}

void commit_scene_data(rt_scene* dst, const rt_scene* src, void* mem) {
    (void)hipSetDevice(dst->device);
    // a different light count changes the shadow queue's size and the node-index limit
    const bool new_lights = dst->n_point_lights != src->n_point_lights || dst->S.n_lights != src->S.n_lights;
    if (dst->dmem) (void)hipFree(dst->dmem);
    dst->dmem = mem;
    dst->dbytes = src->dbytes;
    dst->S = src->S;
    const uint8_t* from = (const uint8_t*)src->dmem;
    uint8_t* to = (uint8_t*)dst->dmem;
    auto rebase = [&](auto& ptr) {
        if (ptr) ptr = reinterpret_cast<std::remove_reference_t<decltype(ptr)>>(to + ((const uint8_t*)ptr - from));
    };
    DevScene& S = dst->S;
    rebase(S.dsph); rebase(S.gsph); rebase(S.tri); rebase(S.cube); rebase(S.plane); rebase(S.cubetri);
    rebase(S.shapes); rebase(S.mats); rebase(S.lights); rebase(S.bvh_nodes); rebase(S.bvh_leaves);
    rebase(S.graze_blk); rebase(S.graze_tri); rebase(S.graze_pn); rebase(S.graze_mask); rebase(S.scan_ops);
    dst->flops_per_scan = src->flops_per_scan;
    dst->normal_max = src->normal_max;
    dst->n_point_lights = src->n_point_lights;
    dst->d_mats = src->d_mats;
    dst->d_shapes = src->d_shapes;
    dst->d_lights = src->d_lights;
    dst->d_ambient = src->d_ambient;
    // deeper ray trees may need a larger pool than any pass checked so far: check again
    dst->checked_items = 0;
    dst->checked_depth = 0;
    // the kernels' LDS staging depends on the scene (node records, grazing normals, sphere
    // pairs): the persistent grids are sized from the occupancy measured again
    dst->occ_trace = 0;
    dst->generation++;
    if (new_lights) free_workspace(dst->ws);
}

}  // namespace

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

rt_status rt_scene_destroy(rt_scene* s) {
    if (!s) return RT_ERR_INVALID_ARG;
    if (s->multi) rt_multi_free(s->multi);
    s->multi = nullptr;
    if (s->split) rt_multi_free(s->split);
    s->split = nullptr;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    for (auto& se : s->ev_streams) (void)hipEventSynchronize(se.second);  // renders on other streams
    free_workspace(s->ws);
    if (s->dmem) (void)hipFree(s->dmem);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    for (auto& se : s->ev_streams) (void)hipEventDestroy(se.second);
    for (hipEvent_t e : s->kt_events) (void)hipEventDestroy(e);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return RT_OK;
}

rt_status rt_host_alloc(uint64_t bytes, void** out) {
    if (!out || bytes == 0) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_ERR_NO_DEVICE;
    HIP_TRY(hipHostMalloc(out, bytes, hipHostMallocPortable));
    return RT_OK;
}

rt_status rt_host_free(void* ptr) {
    if (!ptr) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipHostFree(ptr));
    return RT_OK;
}

uint64_t rt_scene_flops_per_scan(const rt_scene* s) { return s ? s->flops_per_scan : 0; }

uint64_t rt_scene_workspace_bytes(const rt_scene* s) {
    if (!s) return 0;
    const Workspace& w = s->ws;
    uint64_t b = (uint64_t)w.out_floats * 4 + w.out8_bytes + 4 * 8 + 64;
    b += (uint64_t)w.capacity * (sizeof(Task) + 4 + 3 * 16 + 4 * w.lit_words + 2 * 16);  // tasks, node arrays
    if (w.forest) b += (uint64_t)w.capacity * (2 * 16 + 4 + 4);
    b += (uint64_t)w.sort_capacity * 8;                                      // task keys, permutation
    b += (uint64_t)w.shadow_capacity * (w.shadow_light ? 8 : 4) + (uint64_t)w.sort_shadow_capacity * 8;
    b += (uint64_t)w.sort_tmp_words * 4;
    b += (uint64_t)w.spp_buf_floats * 4;
    if (w.levels) b += RT_LEVEL_TABLE_WORDS * 4 + 64;
    return b;
}
uint64_t rt_scene_device_bytes(const rt_scene* s) { return s ? (uint64_t)s->dbytes : 0; }

rt_status rt_scene_scan_ops(rt_scene* s, uint64_t* out, uint32_t n, int32_t reset) {
    if (!s || (out && n > RT_SCAN_OPS_N)) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipDeviceSynchronize());
    if (out && n) {
        std::vector<unsigned long long> h(RT_OPS_SLOTS * RT_OPS_STRIDE);
        HIP_TRY(hipMemcpy(h.data(), s->S.scan_ops, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        for (uint32_t k = 0; k < n; k++) {
            out[k] = 0;
            for (int b = 0; b < RT_OPS_SLOTS; b++) out[k] += h[b * RT_OPS_STRIDE + k];
        }
    }
    if (reset) {
        HIP_TRY(hipMemset(s->S.scan_ops, 0, RT_OPS_SLOTS * RT_OPS_STRIDE * sizeof(unsigned long long)));
        HIP_TRY(hipDeviceSynchronize());
    }
    return RT_OK;
}

int32_t rt_scene_uses_bvh(const rt_scene* s) { return (s && s->S.use_bvh) ? 1 : 0; }

rt_status rt_scene_set_grid_share(rt_scene* s, int32_t percent) {
    if (!s || percent < 1 || percent > 100) return RT_ERR_INVALID_ARG;
    if (s->multi) (void)rt_multi_each(s->multi, [&](rt_scene* c) { return rt_scene_set_grid_share(c, percent); });
    if (s->split) (void)rt_multi_each(s->split, [&](rt_scene* c) { return rt_scene_set_grid_share(c, percent); });
    s->grid_pct = percent;
    return RT_OK;
}

rt_status rt_scene_set_tuning(rt_scene* s, const char* tuning) {
    if (!s) return RT_ERR_INVALID_ARG;
    Tune t = s->tune;
    if (!tune_apply(t, tuning, false)) return RT_ERR_INVALID_ARG;
    auto set = [&](rt_scene* c) {  // clones share the scene-build keys
        c->tune = t;
        c->occ_trace = 0;  // the kernels' LDS may differ: occupancy measured again
        return RT_OK;
    };
    (void)set(s);
    if (s->multi) (void)rt_multi_each(s->multi, set);
    if (s->split) (void)rt_multi_each(s->split, set);
    return RT_OK;
}

rt_status rt_scene_set_scan_counting(rt_scene* s, int32_t enable) {
    if (!s) return RT_ERR_INVALID_ARG;
    if (s->multi) (void)rt_multi_each(s->multi, [&](rt_scene* c) { return rt_scene_set_scan_counting(c, enable); });
    if (s->split) (void)rt_multi_each(s->split, [&](rt_scene* c) { return rt_scene_set_scan_counting(c, enable); });
    s->count_ops = enable != 0;
    return RT_OK;
}

rt_status rt_scene_set_kernel_timing(rt_scene* s, int32_t enable) {
    if (!s) return RT_ERR_INVALID_ARG;
    s->ktime = enable != 0;
    return RT_OK;
}

rt_status rt_scene_kernel_times(rt_scene* s, float* ms, uint32_t n, int32_t reset) {
    if (!s || (n && !ms)) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(s->device));
    for (uint32_t k = 0; k < n; k++) ms[k] = 0.f;
    for (const auto& sp : s->kt_spans) {
        HIP_TRY(hipEventSynchronize(s->kt_events[sp.second + 1]));
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, s->kt_events[sp.second], s->kt_events[sp.second + 1]));
        if ((uint32_t)sp.first < n) ms[sp.first] += t;
    }
    if (n > RT_KT_LAUNCHES) ms[RT_KT_LAUNCHES] = (float)s->kt_spans.size();
    if (reset) {
        s->kt_spans.clear();
        s->kt_used = 0;
    }
    return RT_OK;
}

#if RT_DIAG
static uint32_t* g_task_clock = nullptr;  // RT_TASK_CLOCK records (diagnostic builds)
#endif

// Where one render pass's results go: the float frame (or band buffer), optionally its
// Color::as_u8 bytes (fused into the level-0 combine), ray counters, and whether queue
// overflows are latched into the scene's sticky status (the stream-ordered entry points;
// rt_render retries instead).
struct PassOut {
    float* rgb;
    uint8_t* rgb8;
    unsigned long long* counters;
    bool latch;
    bool may_sync;  // the caller waits anyway (rt_render, forests): deep passes stop at the first empty level
    bool direct = false;  // rgb / rgb8 are whole frames: this rank's rows land in place (row-major)
};

static rt_status launch_bands_wave(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                                   uint32_t band_rows, uint32_t rank, uint32_t world, const PassOut& o,
                                   hipStream_t stream);

static rt_status launch_bands(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                              uint32_t band_rows, uint32_t rank, uint32_t world, const PassOut& o,
                              hipStream_t stream) {
    if (!s || !cam || (!o.rgb && !o.rgb8) || band_rows == 0 || world == 0 || rank >= world) return RT_ERR_INVALID_ARG;
    if (spp == 0) return RT_ERR_INVALID_ARG;
    if (cam->x_res == 0 || cam->y_res == 0) return RT_ERR_INVALID_ARG;
    if (depth > RT_MAX_DEPTH) return RT_ERR_UNSUPPORTED;
    if ((uint64_t)cam->x_res * cam->y_res * 3 >= (1ull << 32)) return RT_ERR_UNSUPPORTED;
    rt_status st = ensure_ws(s, 0, 0);
    if (st != RT_OK) return st;
    return launch_bands_wave(s, cam, depth, spp, seed, band_rows, rank, world, o, stream);
}

// Level-synchronous pipeline: trace(0..L-1), then combine(L-1..0), all on `stream`.
// The level-synchronous pipeline into workspace `w`.  Forest builds (w.forest) write the
// per-node shade inputs, always read the level sizes on the host, skip the combine pass
// and leave the parameters (with the device level table) in *forest_params.
static rt_status wave_pipeline(rt_scene* s, Workspace& w, const rt_camera* cam, uint32_t depth, uint32_t band_rows,
                               uint32_t rank, uint32_t world, const PassOut& o, hipStream_t stream,
                               WaveParams* forest_params, uint32_t* forest_levels, uint32_t spp = 1,
                               uint32_t sample = 0, uint32_t seed = 0, uint32_t frames = 1,
                               const rt_camera* cams = nullptr, bool spp_batch = false,
                               hipEvent_t forest_done = nullptr);

// Samples per pipeline pass for spp > 1: Tune::spp_batch, else as many (<= RT_MAX_FRAMES) as
// keep a pass within Tune::spp_batch_items level-0 items (default 2^25: 4 x 3840x2160 or
// 8 x 1920x1080; the pass's workspace grows with its items).
static uint32_t spp_batch_size(const Tune& tn, uint32_t spp, uint64_t frame_items) {
    if (tn.spp_batch > 0) return (uint32_t)std::max(1, std::min(tn.spp_batch, (int)RT_MAX_FRAMES));
    const uint64_t cap = tn.spp_batch_items;
    uint32_t b = 1;
    while (b < RT_MAX_FRAMES && b < spp && (uint64_t)(b + 1) * frame_items <= cap) b++;
    return b;
}

// spp samples in sample order.  Batched (the default): B samples per pipeline pass, each a
// "frame" of the pass with the same camera and its own jitter (sample index = base + frame),
// its raw colour written to its own buffer; spp_accumulate_kernel then folds the batch into
// the running sum in sample order and the last batch divides -- the same f32 operations as
// one pass per sample, where the level-0 combine adds sample k's colour to the running sum
// of samples 0..k-1 and the last one divides (RT_SPP_BATCH=1).
static rt_status launch_bands_wave(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                                   uint32_t band_rows, uint32_t rank, uint32_t world, const PassOut& o,
                                   hipStream_t stream) {
    const uint32_t rows_local = rt_band_rows_per_rank(cam->y_res, band_rows, world);
    const uint64_t frame_items = (uint64_t)((cam->x_res + 7) / 8) * ((rows_local + 7) / 8) * 64u;
    const uint32_t sb = spp > 1 && o.rgb && (uint64_t)cam->x_res * cam->y_res < (1ull << RT_FRAME_SHIFT)
                            ? spp_batch_size(s->tune, spp, frame_items) : 1u;
    if (sb > 1) {
        Workspace& w = s->ws;
        const size_t frame_floats = (size_t)rows_local * cam->x_res * 3u;
        if (w.spp_buf_floats < sb * frame_floats) {
            if (w.spp_buf) (void)hipFree(w.spp_buf);
            w.spp_buf = nullptr;
            w.spp_buf_floats = 0;
            HIP_TRY(hipMalloc(&w.spp_buf, sb * frame_floats * sizeof(float)));
            w.spp_buf_floats = sb * frame_floats;
        }
        rt_camera cams[RT_MAX_FRAMES];
        for (uint32_t f = 0; f < sb; f++) cams[f] = *cam;
        const PassOut ob{w.spp_buf, nullptr, o.counters, o.latch, o.may_sync};
        for (uint32_t k = 0; k < spp; k += sb) {
            const uint32_t b = std::min(sb, spp - k);
            rt_status st = wave_pipeline(s, w, cam, depth, band_rows, rank, world, ob, stream, nullptr, nullptr, spp, k,
                                         seed, b, cams, true);
            if (st != RT_OK) return st;
            HIP_TRY(launch_spp_accumulate(w.spp_buf, b, frame_floats, k, spp, o.rgb, o.rgb8, stream));
        }
        return RT_OK;
    }
    for (uint32_t k = 0; k < spp; k++) {
        rt_status st = wave_pipeline(s, s->ws, cam, depth, band_rows, rank, world, o, stream, nullptr, nullptr, spp, k,
                                     seed);
        if (st != RT_OK) return st;
    }
    return RT_OK;
}

static rt_status wave_pipeline(rt_scene* s, Workspace& w, const rt_camera* cam, uint32_t depth, uint32_t band_rows,
                               uint32_t rank, uint32_t world, const PassOut& o, hipStream_t stream,
                               WaveParams* forest_params, uint32_t* forest_levels, uint32_t spp, uint32_t sample,
                               uint32_t seed, uint32_t frames, const rt_camera* cams, bool spp_batch,
                               hipEvent_t forest_done) {
    if (frames == 0 || frames > RT_MAX_FRAMES || (frames > 1 && (!cams || forest_params))) return RT_ERR_INVALID_ARG;
    WaveParams p;
    std::memset(&p, 0, sizeof(p));
    p.spp = spp;
    p.spp_batch = spp_batch ? 1u : 0u;
    // queue keys of a sample batch: "mix" -- no sample index in the keys, the samples of one
    // place share waves; "mixfine" (default) -- the same with a frame batch's finer 21-bit
    // task / 4-bit-distance shadow keys; "frame" -- the sample index above the key bits like
    // a frame batch (Tune::spp_keys, A/B)
    // (frame batches: Tune::frame_keys, default "mixfine" as well)
    // measured (config 5, 4 passes of 4K x 64 samples in batches of 4): mix 1021, mixfine
    // 1058, frame 1023 Msamples/s; one pass per sample 788.  Frame batches (config 3, 4 passes
    // of 5 frames): frame 944 / 945, mix 1023 / 1018, mixfine 1073 / 1076 Mpixels/s with one
    // camera for every frame; with a camera per frame (an animation) frame 948, mixfine 1025
    const Tune& tn = s->tune;
    const int spp_keys = spp_batch ? tn.spp_keys : tn.frame_keys;
    p.frame_keys = spp_keys == 2 ? 1u : 0u;
    {
        // level-0 tiles dealt to a pass's frames in turn (default since the 16-frame passes:
        // 1124 - 1133 vs 1116 - 1122 Mpixels/s in 7 alternating pairs, tools/r3_ab23.sh /
        // r3_ab24.sh; at 5-frame passes it was noise); l0_interleave=0: frame-major (A/B)
        p.l0_interleave = tn.l0_interleave ? 1u : 0u;
    }
    p.sample = sample;
    p.seed = seed;
    p.S = s->S;
    p.width = cam->x_res;
    p.height = cam->y_res;
    p.depth = depth;
    p.band_rows = band_rows;
    p.rank = rank;
    p.world = world;
    p.rows_local = rt_band_rows_per_rank(cam->y_res, band_rows, world);
    p.tiles_x = (cam->x_res + 7) / 8;
    uint64_t total = (uint64_t)p.tiles_x * ((p.rows_local + 7) / 8) * 64u;
    p.frames = frames;
    p.frame_items = (uint32_t)total;
    p.frame_floats = (size_t)p.rows_local * p.width * 3u;
    if (o.direct) {
        if (spp_batch || forest_params) return RT_ERR_INVALID_ARG;
        p.direct = 1u;
        p.frame_floats = (size_t)p.height * p.width * 3u;
    }
    if (frames > 1 && (uint64_t)cam->x_res * cam->y_res >= (1ull << RT_FRAME_SHIFT)) return RT_ERR_UNSUPPORTED;
    {
        // level 0 reads every frame's camera from cams[] (frames == 1: cams[0] = cam)
        if (frames == 1) cams = cam;
        for (uint32_t f = 0; f < frames; f++) {
            if (cams[f].x_res != cam->x_res || cams[f].y_res != cam->y_res) return RT_ERR_INVALID_ARG;
            FrameCam& c = p.cams[f];
            c.ox = cams[f].origin[0];
            c.oy = cams[f].origin[1];
            c.oz = cams[f].origin[2];
            c.x_min = cams[f].x_min;
            c.y_max = cams[f].y_max;
            c.x_delta = (cams[f].x_max - cams[f].x_min) / (float)cams[f].x_res;  // render.rs:179-180
            c.y_delta = (cams[f].y_max - cams[f].y_min) / (float)cams[f].y_res;
            c.pad = 0.f;
        }
    }
    total *= frames;
    if (total >= (1ull << 30)) return RT_ERR_UNSUPPORTED;
    p.total_items = (uint32_t)total;
    // node / task pool: Tune::node_factor (default 6) nodes per level-0 item -- config 3
    // traces 3.66 node rays per pixel, config 4 the same scene at 4K; an overflow is
    // reported, never silently truncated, and the next pass gets twice the pool (rt_render
    // retries by itself).  A shadow entry packs (node << light_bits) | light, so nodes stay
    // below 2^(32 - light_bits).
    p.light_bits = light_bits(s);
    const uint64_t max_cap = pool_cap_limit(s);
    if (total >= max_cap) return RT_ERR_UNSUPPORTED;
    uint64_t want = std::max<uint64_t>(total * (uint64_t)tn.node_factor, 1u << 20);
    if (tn.node_cap) want = std::max<uint64_t>(total + 1, tn.node_cap);  // test knob
    if (&w == &s->ws) want = std::max<uint64_t>(want, s->pool_floor);
    if (want > max_cap) want = max_cap;
    const uint32_t lit_words = ((uint32_t)s->S.n_lights + 31u) / 32u > 1u ? ((uint32_t)s->S.n_lights + 31u) / 32u : 1u;
    if (w.capacity < want || w.lit_words != lit_words) {  // grows only (rt_render may have grown it after an overflow)
        w.lit_words = lit_words;
        rt_status st = grow_node_pool(w, (uint32_t)std::max<uint64_t>(want, w.capacity));
        if (st != RT_OK) return st;
    }
    if (!w.levels) {
        HIP_TRY(hipMalloc(&w.levels, RT_LEVEL_TABLE_WORDS * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&w.overflow, 64));
        // stream-ordered on the pass's own stream: a hipMemset on the null stream is not
        // ordered with the caller's non-blocking stream and could land after this pass had
        // latched an overflow (profiles/r3y: a missed RT_ERR_CAPACITY that depended on which
        // hardware queue the null stream shared with another slot's pass)
        HIP_TRY(hipMemsetAsync(w.overflow, 0, 64, stream));
    }
    // shadow queue: at most one entry per point light per hit node; Tune::shadow_factor
    // (default 2) entries per node slot, at most the point lights (config 3 queues 2.0 per
    // traced node: the trace kernel decides the rest; overflow reported like the node pool's)
    // Scenes of more than 32 point lights: lights 32 and up are never decided by the trace
    // kernel, so a hit queues about one entry per point light -- the queue is sized for that
    const double sh_per_node = s->n_point_lights > 32u ? (double)s->n_point_lights
                                                        : std::min<double>(tn.shadow_factor, (double)s->n_point_lights);
    uint64_t want_sh = std::min<uint64_t>((uint64_t)((double)w.capacity * sh_per_node), 0x7FFFFFFFu);
    if (want_sh == 0) want_sh = 1;
    const bool wide = wide_entries(s);
    if (w.shadow_capacity < want_sh || wide != (w.shadow_light != nullptr)) {
        for (uint32_t** b : {&w.shadow, &w.shadow_light}) {
            if (*b) (void)hipFree(*b);
            *b = nullptr;
        }
        want_sh = std::max<uint64_t>(want_sh, w.shadow_capacity);
        w.shadow_capacity = 0;
        HIP_TRY(hipMalloc(&w.shadow, want_sh * sizeof(uint32_t)));
        if (wide) HIP_TRY(hipMalloc(&w.shadow_light, want_sh * sizeof(uint32_t)));
        w.shadow_capacity = (uint32_t)want_sh;
    }
    const bool sort_tasks = s->S.use_bvh && tn.sort_tasks;
    const bool sort_shadow = s->S.use_bvh && tn.sort_shadow;
    p.key_mode = (uint32_t)tn.task_key;
    p.key_ahead = p.key_mode == 5 ? 0.5f : 0.25f;
    p.self_shadow = tn.self_shadow ? 1u : 0u;
    // tracing a level's sorted queue from its end (939 / 947 vs 944 / 945 Mpixels/s) and the
    // dynamic per-wave work counter (6.7 vs 4.9 ms) lost: levels run in queue order, grid-stride
    p.reverse_levels = 0u;
    p.sched = 0u;
    // primary hits are coherent (8x8 tiles): their shadow rays are traced inline by the
    // trace kernel (config 3: -2%); deeper levels' hit points are scattered and go
    // through the sorted shadow queue (inlining levels 0-1: +20%, all: x2.4)
    p.inline_levels = (uint32_t)tn.inline_shadow;
#if RT_DIAG
    {
        // debug: per wave-iteration wall-clock records of the trace kernel (rt_debug_task_clock)
        static uint32_t* clk = nullptr;
        static uint32_t clk_cap = 0;
        const char* e = std::getenv("RT_TASK_CLOCK");
        if (e && !clk) {
            clk_cap = (uint32_t)std::atoi(e);
            HIP_TRY(hipMalloc(&clk, (4 + 4 * (size_t)clk_cap) * sizeof(uint32_t)));
            g_task_clock = clk;
        }
        p.task_clock = e ? clk : nullptr;
        p.task_clock_cap = clk_cap;
        if (p.task_clock) HIP_TRY(hipMemsetAsync(p.task_clock, 0, 16, stream));
    }
#else
    p.task_clock = nullptr;
    p.task_clock_cap = 0;
#endif
    // narrowest trace task width (64: fixed 64-ray tasks) and the tasks per wave slot below
    // which a level's tasks are narrowed
    p.task_w_min = (uint32_t)tn.task_w;
    p.task_w_fill = (float)tn.task_fill;
    // instrumented kernels (counting frames): Tune::count selects the kernels that count
    p.count_mask = s->count_ops ? (uint32_t)tn.count : 0u;
    p.lds_mask = (uint32_t)tn.lds_nodes;
    p.deep_kernel = (uint32_t)tn.deep_kernel;
    p.occ_each = (uint32_t)tn.occ_each;
    // 16-bit keys: task = direction cell | coarse origin Morton (task_key); shadow =
    // light index | the Morton bits that fit (all 15 above 16 lights' worth of bits)
    uint32_t lbits = 0;
    while ((1u << lbits) < s->S.n_lights) lbits++;
    p.light_shift = lbits <= 1 ? 15u : (16u - lbits > 15u ? 15u : 16u - lbits);
    uint32_t task_bits = (p.key_mode == 3 || p.key_mode == 4) ? 24u : 16u, shadow_bits = 16u;
    {
        // light | light-buffer cell | 3-bit distance from the light by default ("cell2": a wave
        // holds rays that test one cell's records, at similar reach; rays that walk the
        // hierarchy: light | flag | 17-bit Morton): 790 / 789 Mpixels/s vs 784 / 775 for the
        // cell alone ("cell") and 752 / 763 for light | 18-bit Morton ("18", round 1's
        // default; round 1: 4.80 ms vs 4.93 with the 16-bit key "16"); Tune::shadow_key (A/B)
        const uint32_t cell = tn.shadow_key == 1 ? 1u : (tn.shadow_key == 2 ? 2u : 0u);
        const int v = cell ? 18 : tn.shadow_key;
        p.shadow_fine = (p.key_mode == 3 || p.key_mode == 4 || v == 18) ? 18u : (v == 21 ? 21u : 0u);
        if (p.shadow_fine && p.shadow_fine + lbits > 32u) p.shadow_fine = 0u;
        // cell keys: the light-buffer cell index (x 8 distance buckets for cell2) must fit
        // below the flag bit
        const uint64_t cells = 6ull * s->S.lb_res * s->S.lb_res * (cell == 2u ? 8u : 1u);
        p.shadow_cell = (cell && p.shadow_fine == 18u && s->S.lb_res && cells < (1u << 17)) ? cell : 0u;
    }
    if (p.shadow_fine) shadow_bits = p.shadow_fine + lbits;
    // (one frame with a batch's finer keys -- 21-bit task keys, 4-bit shadow distance --
    // measured 4.08 vs 4.11 ms, split 3.88 vs 3.76: not kept)
    if (frames > 1 && spp_keys != 0) {  // the frame index above every key bit: frames are contiguous in sorted queues (ordering only)
        uint32_t fbits = 0;
        while ((1u << fbits) < frames) fbits++;
        if (!p.frame_keys) fbits = 0;  // "mixfine": the finer keys without the sample index
        // a batch's task keys take 3 radix passes of 8 bits anyway: key mode 7 fills them with
        // 5 more origin bits (task_fine=0: off, A/B)
        if (tn.task_fine && p.key_mode == 7 && task_bits == 16u && fbits <= 3) {
            p.task_fine = 1u;
            task_bits = 21u;
        }
        // ... and the shadow keys a fourth distance bit when 3 passes still hold them
        // (shadow_fine=0: off, A/B)
        if (tn.shadow_fine && p.shadow_cell == 2u && p.shadow_fine == 18u && shadow_bits + 1u + fbits <= 24u &&
            6ull * s->S.lb_res * s->S.lb_res * 16u < (1u << 18)) {
            p.shadow_cell = 3u;
            p.shadow_fine = 19u;
            shadow_bits += 1u;
        }
        // without frame bits a batch's 3 radix passes hold 24 key bits: 18-bit Morton task keys
        // and a 7-bit shadow distance (1035 / 1039 vs 1027 / 1031 Mpixels/s with the 21-bit
        // keys; key24=0: off, A/B; 4x4 direction cells | 16-bit Morton instead: no gain)
        if (tn.key24 && fbits == 0) {
            if (p.task_fine == 1u) {
                p.task_fine = 2u;
                task_bits = 24u;
            }
            if (p.shadow_cell == 3u && 6ull * s->S.lb_res * s->S.lb_res * 128u < (1u << 21) && lbits + 22u <= 24u) {
                p.shadow_cell = 4u;
                p.shadow_fine = 22u;
                shadow_bits = 22u + lbits;
            }
        }
        p.task_frame_shift = task_bits;
        p.shadow_frame_shift = shadow_bits;
        task_bits += fbits;
        shadow_bits += fbits;
        if (shadow_bits > 32u) return RT_ERR_UNSUPPORTED;
    }
    if (sort_tasks && w.sort_capacity < w.capacity) {
        for (uint32_t** b : {&w.task_keys, &w.perm}) {
            if (*b) (void)hipFree(*b);
            *b = nullptr;
        }
        w.sort_capacity = 0;
        for (uint32_t** b : {&w.task_keys, &w.perm}) HIP_TRY(hipMalloc(b, (size_t)w.capacity * sizeof(uint32_t)));
        w.sort_capacity = w.capacity;
    }
    if (sort_shadow && w.sort_shadow_capacity < w.shadow_capacity) {
        for (uint32_t** b : {&w.shadow_keys, &w.shadow_sorted}) {
            if (*b) (void)hipFree(*b);
            *b = nullptr;
        }
        w.sort_shadow_capacity = 0;
        for (uint32_t** b : {&w.shadow_keys, &w.shadow_sorted})
            HIP_TRY(hipMalloc(b, (size_t)w.shadow_capacity * sizeof(uint32_t)));
        w.sort_shadow_capacity = w.shadow_capacity;
    }
    // sort scratch: keys + values for the larger queue, its tile counts, digit totals
    const uint32_t sort_cap = std::max(w.capacity, w.shadow_capacity);
    const size_t sort_words =
        4 * (size_t)sort_cap + (size_t)sort_max_digits() * sort_max_tiles(sort_cap) + sort_max_digits();
    if ((sort_tasks || sort_shadow) && w.sort_tmp_words < sort_words) {
        if (w.sort_tmp) (void)hipFree(w.sort_tmp);
        w.sort_tmp = nullptr;
        w.sort_tmp_words = 0;
        HIP_TRY(hipMalloc(&w.sort_tmp, sort_words * sizeof(uint32_t)));
        w.sort_tmp_words = sort_words;
    }
    uint32_t* sort_scratch = w.sort_tmp;
    uint32_t* tile_counts = w.sort_tmp ? w.sort_tmp + 4 * (size_t)sort_cap : nullptr;
    uint32_t* digit_totals = w.sort_tmp ? tile_counts + (size_t)sort_max_digits() * sort_max_tiles(sort_cap) : nullptr;
    // radix digits of up to RT_SORT_DIGIT (8..11) bits, the fewest passes for the key: 8 by
    // default (byte digits: 3 passes for the 17-bit task keys of a 2-frame batch and the
    // 21-bit shadow keys).  At 4 passes x 2 frames in flight: 9 (task keys in 2 passes)
    // 788 / 795 vs 791 / 790 Mpixels/s, 11 (every key in 2 passes) 751 / 750 vs 789 / 785 --
    // a wider digit's ranking and tile counts cost more than the pass it saves
    const uint32_t sort_digit = 8u;
    p.task_keys = sort_tasks ? w.task_keys : nullptr;
    p.perm = nullptr;
    p.shadow_keys = sort_shadow ? w.shadow_keys : nullptr;
    // packed entries are read straight from the queue; wide ones by slot (null: slot t)
    p.shadow_in = wide ? nullptr : w.shadow;
    p.shadow_light = w.shadow_light;
    p.capacity = w.capacity;
    p.shadow_capacity = w.shadow_capacity;
    p.shadow = w.shadow;
    p.tasks = w.tasks;
    p.node_flags = w.node_flags;
    p.node_ps = w.node_ps;
    p.node_n = w.node_n;
    p.node_d = w.node_d;
    p.node_lit = w.node_lit;
    p.node_lit_hi = w.node_lit_hi;
    p.lit_words = w.lit_words;
    p.node_ec = w.node_ec;
    p.levels = w.levels;
    p.overflow = w.overflow;
    p.overflow_sticky = o.latch ? w.overflow + 1 : nullptr;
    p.out = o.rgb;
    p.out8 = o.rgb8;
    p.ray_counters = o.counters;
    if (w.forest) {
        p.node_dc = w.node_dc;
        p.node_key = w.node_key;
        p.node_pixel = w.node_pixel;
    }
    if (s->occ_trace == 0) {
        int a = 0, b = 0, c = 0;
        HIP_TRY(wave_occupancy(p, &a, &b, &c, s->occ_trace_each));
        s->occ_trace = a > 0 ? a : 1;
        s->occ_shadow = b > 0 ? b : 1;
        s->occ_combine = c > 0 ? c : 1;
    }
    int tb = s->num_cus * s->occ_trace;
    int sb = s->num_cus * s->occ_shadow;
    int cb = s->num_cus * s->occ_combine;
    {
        // the persistent trace grids at grid_pct % of a full chip (rt_scene_set_grid_share;
        // Tune::grid_pct overrides it, A/B)
        const int pct = tn.grid_pct ? tn.grid_pct : s->grid_pct;
        // the shadow pass keeps the whole chip (measured: 937 vs 927 Mpixels/s at 75%);
        // Tune::grid_pct_shadow sets its own share (A/B)
        const int spct = tn.grid_pct_shadow;
        if (pct > 0 && pct < 100) tb = std::max(1, tb * pct / 100);
        if (spct > 0 && spct < 100) sb = std::max(1, sb * spct / 100);
        // the combine grids too (50% / 25%: 928 / 918, 889 / 896 vs 936 / 940 Mpixels/s);
        // Tune::grid_pct_combine (A/B)
        const int cpct = tn.grid_pct_combine;
        if (cpct > 0 && cpct < 100) cb = std::max(1, cb * cpct / 100);
    }
    uint32_t levels = depth > 0 ? depth : 1;
    // measurement (Tune::dup, letters s / h / c): launch every queue sort / the shadow pass /
    // every combine twice -- each is idempotent -- to measure a stage's marginal cost in place
    const int dup_sort = (tn.dup & 1) ? 2 : 1, dup_shadow = (tn.dup & 2) ? 2 : 1, dup_comb = (tn.dup & 4) ? 2 : 1;
    // Every launch sizes itself from the device-side level counts: the whole frame is
    // enqueued without a host round trip (levels past the deepest non-empty one are no-ops).
    HIP_TRY(launch_wave_init(w.levels, RT_LEVEL_TABLE_WORDS, p.total_items, sample == 0 ? w.overflow : nullptr,
                             stream));
    if (w.lit_words > 1)  // lights 32 and up: their bits start at 0 (the trace kernel stores word 0 only)
        HIP_TRY(hipMemsetAsync(w.node_lit_hi, 0, (size_t)(w.lit_words - 1) * w.capacity * sizeof(uint32_t), stream));
    {
        KSpan k0(s, stream, RT_KT_TRACE);
        HIP_TRY(launch_wave_trace(p, 0, tb, stream, s->occ_trace_each, s->occ_trace));
    }
    // every level's queue is sorted (leaving any level unsorted lost: DESIGN.md)
    const uint64_t sort_levels = ~0ull;
    for (uint32_t k = 1; k < levels; k++) {
        if (o.may_sync && levels > 16 && (k & 7u) == 0) {
            // a deep pass the caller waits for anyway: stop at the first empty level (the
            // levels after it would be no-op launches; the ray trees have ended)
            uint32_t next = 0;
            HIP_TRY(hipMemcpyAsync(&next, w.levels + 2 * k + 1, sizeof(next), hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            if (next == 0) {
                levels = k;
                break;
            }
        }
        p.perm = nullptr;  // production order unless this level is sorted
        if (sort_tasks && ((sort_levels >> (k < 64 ? k : 63)) & 1ull)) {
            KSpan ks(s, stream, RT_KT_SORT_TASKS);
            for (int r = 0; r < dup_sort; r++)
                HIP_TRY(launch_sort(w.levels, (int32_t)k, w.capacity, task_bits, w.task_keys, nullptr, sort_scratch,
                                    w.perm, tile_counts, digit_totals, 4 * s->num_cus, stream, sort_digit));
            p.perm = w.perm;
        }
        KSpan kt(s, stream, RT_KT_TRACE);
        HIP_TRY(launch_wave_trace(p, k, tb, stream, s->occ_trace_each, s->occ_trace));
    }
    if (sort_shadow) {
        KSpan ks(s, stream, RT_KT_SORT_SHADOW);
        for (int r = 0; r < dup_sort; r++)
            HIP_TRY(launch_sort(w.levels, -1, w.shadow_capacity, shadow_bits, w.shadow_keys, wide ? nullptr : w.shadow,
                                sort_scratch, w.shadow_sorted, tile_counts, digit_totals, 4 * s->num_cus, stream,
                                sort_digit));  // (wide entries: the values are the slots)
        p.shadow_in = w.shadow_sorted;
    }
    {
        KSpan ksh(s, stream, RT_KT_SHADOW);
        for (int r = 0; r < dup_shadow; r++) HIP_TRY(launch_wave_shadow(p, sb, stream));
    }
    if (w.forest) {  // no combine: the forest is shaded later, any number of times
        if (forest_done) HIP_TRY(hipEventRecord(forest_done, stream));
        HIP_TRY(hipMemcpyAsync(forest_levels, w.levels, 2 * (RT_MAX_DEPTH + 1) * sizeof(uint32_t),
                               hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        uint32_t used = 1;  // levels that hold nodes
        for (uint32_t k = 1; k < levels; k++) {
            uint32_t off = forest_levels[2 * k], cnt = forest_levels[2 * k + 1];
            if (off >= w.capacity || std::min(cnt, w.capacity - off) == 0) break;
            used = k + 1;
        }
        p.perm = nullptr;
        *forest_params = p;
        forest_levels[2 * (RT_MAX_DEPTH + 1)] = used;
        return RT_OK;
    }
    for (uint32_t k = levels; k-- > 0;) {
        KSpan kc(s, stream, RT_KT_COMBINE);
        for (int r = 0; r < dup_comb; r++) HIP_TRY(launch_wave_combine(p, k, cb, stream));
    }
    return RT_OK;
}

static rt_status render_bands_impl(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames, uint32_t depth,
                                   uint32_t spp, uint32_t seed, uint32_t band_rows, uint32_t rank, uint32_t world,
                                   float* d_rgb, uint8_t* d_rgb8, uint64_t* d_counters, void* stream, bool direct) {
    rt_scene* s = const_cast<rt_scene*>(scene);
    if (!s || !cams || n_frames == 0 || n_frames > RT_MAX_FRAMES || spp == 0) return RT_ERR_INVALID_ARG;
    if (!d_rgb && (!d_rgb8 || spp > 1)) return RT_ERR_INVALID_ARG;  // spp > 1 accumulates in d_rgb
    if (n_frames > 1 && spp != 1) return RT_ERR_INVALID_ARG;
    const rt_camera* cam = cams;
    if (band_rows == 0 || world == 0 || rank >= world) return RT_ERR_INVALID_ARG;
    if (cam->x_res == 0 || cam->y_res == 0) return RT_ERR_INVALID_ARG;
    if (depth > RT_MAX_DEPTH) return RT_ERR_UNSUPPORTED;
    if ((uint64_t)cam->x_res * cam->y_res * 3 >= (1ull << 32)) return RT_ERR_UNSUPPORTED;
    HIP_TRY(hipSetDevice(s->device));
    rt_status st = ensure_ws(s, 0, 0);
    if (st != RT_OK) return st;
    hipStream_t hs = (hipStream_t)stream;
    const PassOut o{d_rgb, d_rgb8, reinterpret_cast<unsigned long long*>(d_counters), true, false, direct};
    // A pass larger (level-0 items) or deeper than any this handle has completed is checked
    // before the call returns: the pool is sized from node_factor, which suits config-3-like
    // trees, and a mirror- or glass-heavy scene needs more.  The call waits for that pass, and
    // if a queue overflowed it grows the pool and renders it again (the caller's counters
    // restored first), as rt_render does -- so a new scene or frame size costs one
    // synchronisation, not an incomplete frame.  Passes no larger than a checked one stay
    // asynchronous: an overflow there (trees that grew with the camera) is latched and
    // reported by rt_scene_sync_status, and the next pass gets twice the pool.  The node_cap
    // test knob pins the pools and skips the check.
    const uint64_t rows_local = rt_band_rows_per_rank(cam->y_res, band_rows, world);
    const uint64_t items = (uint64_t)((cam->x_res + 7u) / 8u) * ((rows_local + 7u) / 8u) * 64u * n_frames *
                           std::min<uint32_t>(spp, RT_MAX_FRAMES);
    const bool checked = !s->tune.node_cap && (items > s->checked_items || depth > s->checked_depth);
    if (checked) {
        // the check waits on the host: never inside a stream capture (rt_api.h "HOST WAIT")
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        HIP_TRY(hipStreamIsCapturing(hs, &cap));
        if (cap != hipStreamCaptureStatusNone) return RT_ERR_UNSUPPORTED;
        HIP_TRY(hipStreamSynchronize(hs));
        for (auto& se : s->ev_streams) HIP_TRY(hipEventSynchronize(se.second));
        if (s->ws.overflow) {  // an earlier pass's unreported overflow stays reported
            uint32_t v = 0;
            HIP_TRY(hipMemcpyAsync(&v, s->ws.overflow + 1, sizeof(v), hipMemcpyDeviceToHost, hs));
            HIP_TRY(hipStreamSynchronize(hs));
            if (v) {
                s->ovf_pending = true;
                HIP_TRY(hipMemsetAsync(s->ws.overflow + 1, 0, sizeof(v), hs));
            }
        }
        if (d_counters) HIP_TRY(hipMemcpyAsync(s->ws.ctr_save, d_counters, 3 * sizeof(uint64_t), hipMemcpyDeviceToDevice, hs));
    }
    for (int attempt = 0;; attempt++) {
        if (n_frames == 1) {
            st = launch_bands(s, cam, depth, spp, seed, band_rows, rank, world, o, hs);
        } else {
            st = wave_pipeline(s, s->ws, cam, depth, band_rows, rank, world, o, hs, nullptr, nullptr, 1, 0, 0,
                               n_frames, cams);
        }
        if (st != RT_OK || !checked) break;
        uint32_t ovf = 0;
        HIP_TRY(hipMemcpyAsync(&ovf, s->ws.overflow, sizeof(ovf), hipMemcpyDeviceToHost, hs));
        HIP_TRY(hipStreamSynchronize(hs));
        if (!ovf) {
            s->checked_items = std::max(s->checked_items, items);
            s->checked_depth = std::max(s->checked_depth, depth);
            break;
        }
        const uint64_t lim = pool_cap_limit(s);
        if (attempt >= 8 || s->ws.capacity >= lim) break;  // latched: rt_scene_sync_status reports it
        HIP_TRY(hipMemsetAsync(s->ws.overflow + 1, 0, sizeof(uint32_t), hs));  // rendered again
        s->pool_floor = (uint32_t)std::min<uint64_t>(2ull * s->ws.capacity, lim);
        if (d_counters)
            HIP_TRY(hipMemcpyAsync(d_counters, s->ws.ctr_save, 3 * sizeof(uint64_t), hipMemcpyDeviceToDevice, hs));
    }
    if (st != RT_OK) return st;
    hipEvent_t ev = nullptr;
    for (size_t i = 0; i < s->ev_streams.size();) {  // drop completed renders of other streams
        auto& se = s->ev_streams[i];
        if (se.first != hs && hipEventQuery(se.second) == hipSuccess) {
            (void)hipEventDestroy(se.second);
            se = s->ev_streams.back();
            s->ev_streams.pop_back();
            continue;
        }
        if (se.first == hs) ev = se.second;
        i++;
    }
    if (!ev) {
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        s->ev_streams.emplace_back(hs, ev);
    }
    HIP_TRY(hipEventRecord(ev, hs));
    return RT_OK;
}

rt_status rt_render_bands_ex_async(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames, uint32_t depth,
                                   uint32_t spp, uint32_t seed, uint32_t band_rows, uint32_t rank, uint32_t world,
                                   float* d_rgb, uint8_t* d_rgb8, uint64_t* d_counters, void* stream) {
    return render_bands_impl(scene, cams, n_frames, depth, spp, seed, band_rows, rank, world, d_rgb, d_rgb8, d_counters,
                             stream, false);
}

// This rank's rows of n_frames whole frames, written in place (include/rt_api.h): several
// band shares of one device fill the same frames side by side with no assembly step
rt_status rt_render_bands_direct_async(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames,
                                       uint32_t depth, uint32_t band_rows, uint32_t rank, uint32_t world,
                                       float* d_frames, uint8_t* d_frames8, uint64_t* d_counters, void* stream) {
    return render_bands_impl(scene, cams, n_frames, depth, 1, 0, band_rows, rank, world, d_frames, d_frames8,
                             d_counters, stream, true);
}

rt_status rt_render_bands_spp_async(const rt_scene* scene, const rt_camera* cam, uint32_t depth, uint32_t spp,
                                    uint32_t seed, uint32_t band_rows, uint32_t rank, uint32_t world, float* d_rgb,
                                    uint64_t* d_counters, void* stream) {
    if (!d_rgb) return RT_ERR_INVALID_ARG;
    return rt_render_bands_ex_async(scene, cam, 1, depth, spp, seed, band_rows, rank, world, d_rgb, nullptr,
                                    d_counters, stream);
}

rt_status rt_render_bands_batch_async(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames,
                                      uint32_t depth, uint32_t band_rows, uint32_t rank, uint32_t world,
                                      float* d_rgb, uint64_t* d_counters, void* stream) {
    if (!d_rgb) return RT_ERR_INVALID_ARG;
    return rt_render_bands_ex_async(scene, cams, n_frames, depth, 1, 0, band_rows, rank, world, d_rgb, nullptr,
                                    d_counters, stream);
}

rt_status rt_render_bands_async(const rt_scene* scene, const rt_camera* cam, uint32_t depth,
                                uint32_t band_rows, uint32_t rank, uint32_t world, float* d_rgb,
                                uint64_t* d_counters, void* stream) {
    return rt_render_bands_spp_async(scene, cam, depth, 1, 0, band_rows, rank, world, d_rgb, d_counters, stream);
}

// rt_render's band shares on this device: s->split with n ranks (s itself and n - 1 clones,
// each rank its own stream); built on first use, rebuilt when n changes
static rt_status ensure_split(rt_scene* s, int n) {
    if (s->split_n == n && s->split) return RT_OK;
    if (s->split) rt_multi_free(s->split);
    s->split = nullptr;
    s->split_n = 0;
    s->split_dev_pending = false;
    std::vector<int32_t> devs((size_t)n, s->device);
    rt_status st = rt_multi_build(s, devs.data(), (uint32_t)n, false, &s->split);
    if (st != RT_OK) return st;
    const bool count = s->count_ops;
    (void)rt_multi_each(s->split, [&](rt_scene* c) { return rt_scene_set_scan_counting(c, count); });
    s->split_n = n;
    s->split_dev_y = 0;
    return RT_OK;
}

// rt_render's seam split in stream order (rt_multi.cpp rt_multi_render_frame_async): the
// frame's top rows [0, rows) and the rest render side by side as two band shares of this
// device -- rt_render's shares (s->split: this handle and one clone, each share on the
// state's own stream; the same two streams as rt_render, since streams created later may
// share a hardware queue: 5.4 vs 3.4 ms for a frame when they did) -- forked from and
// joined back into `stream`.  The meeting row starts at the
// even split and, whenever the previous call's share spans have already completed when the
// next call is enqueued, moves 8 rows toward the share that finished first (within [half,
// 3/4] of the frame); the shares' persistent grids take Tune::seam_grid_pct (default 80) % of
// the chip, or the scene's own share if smaller.  seam_split=1 (or frames under 32 rows):
// one pass on `stream`.  No pixel depends on any of it.
rt_status rt_render_frame_async(const rt_scene* scene, const rt_camera* cam, uint32_t depth, float* d_rgb,
                                uint8_t* d_rgb8, uint64_t* d_counters, void* stream) {
    rt_scene* s = const_cast<rt_scene*>(scene);
    if (!s || !cam || !d_rgb || cam->x_res == 0 || cam->y_res == 0) return RT_ERR_INVALID_ARG;
    if (s->multi) return RT_ERR_UNSUPPORTED;  // a multi-device scene renders through rt_render
    if (depth > RT_MAX_DEPTH) return RT_ERR_UNSUPPORTED;
    if ((uint64_t)cam->x_res * cam->y_res * 3 >= (1ull << 32)) return RT_ERR_UNSUPPORTED;
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t hs = (hipStream_t)stream;
    const uint32_t y = cam->y_res;
    if (s->tune.seam_split != 2 || y < 32u) {
        // one pass: one band of 8-row tiles holding every row, padded to a multiple of 8
        const size_t n = (size_t)cam->x_res * y * 3;
        const size_t n_pad = (size_t)cam->x_res * rt_band_rows_per_rank(y, 8, 1) * 3;
        if (n_pad == n)
            return rt_render_bands_ex_async(s, cam, 1, depth, 1, 0, 8, 0, 1, d_rgb, d_rgb8, d_counters, stream);
        rt_status st = ensure_ws(s, n_pad, d_rgb8 ? n_pad : 0);
        if (st != RT_OK) return st;
        st = rt_render_bands_ex_async(s, cam, 1, depth, 1, 0, 8, 0, 1, s->ws.out, d_rgb8 ? s->ws.out8 : nullptr,
                                      d_counters, stream);
        if (st != RT_OK) return st;
        HIP_TRY(hipMemcpyAsync(d_rgb, s->ws.out, n * sizeof(float), hipMemcpyDeviceToDevice, hs));
        if (d_rgb8) HIP_TRY(hipMemcpyAsync(d_rgb8, s->ws.out8, n, hipMemcpyDeviceToDevice, hs));
        return RT_OK;
    }
    rt_status st0 = ensure_split(s, 2);
    if (st0 != RT_OK) return st0;
    const uint32_t even = ((y + 1u) / 2u + 7u) / 8u * 8u;
    const uint32_t hi = std::max(even, (y * 3u / 4u) / 8u * 8u);
    if (s->split_dev_y != y || s->split_dev_rows < even || s->split_dev_rows > hi) {
        s->split_dev_rows = even;
        s->split_dev_y = y;
        // both shares' node pools sized once for the largest share they can get (unless the
        // node_cap test knob pins them)
        const uint64_t floor = std::min<uint64_t>((uint64_t)hi * cam->x_res * (uint64_t)s->tune.node_factor,
                                                  pool_cap_limit(s));
        if (!s->tune.node_cap)
            (void)rt_multi_each_rank(s->split, [&](rt_scene* c) {
                c->pool_floor = std::max<uint32_t>(c->pool_floor, (uint32_t)floor);
                return RT_OK;
            });
    } else {
        float t[2] = {0.f, 0.f};
        if (rt_multi_async_share_ms(s->split, t, 2) == RT_OK && t[0] > 0.f && t[1] > 0.f) {
            const float late = t[1] - t[0], band = 0.03f * t[1];  // > 0: share 0 can take more rows
            if (late > band && s->split_dev_rows + 8u <= hi)
                s->split_dev_rows += 8u;
            else if (late < -band && s->split_dev_rows >= even + 8u)
                s->split_dev_rows -= 8u;
        }
    }
    const int pct = std::min(s->grid_pct, s->tune.seam_grid_pct);
    const int saved = s->grid_pct;  // read when the passes are enqueued: restored right after
    auto set_pct = [&](int v) {
        s->grid_pct = v;
        (void)rt_multi_each(s->split, [&](rt_scene* c) {
            c->grid_pct = v;
            return RT_OK;
        });
    };
    set_pct(pct);
    rt_status st = rt_multi_render_frame_async(s->split, cam, depth, s->split_dev_rows, d_rgb, d_rgb8, d_counters, hs);
    set_pct(saved);
    if (st != RT_OK) return st;
    s->split_dev_pending = true;
    return RT_OK;
}

rt_status rt_scene_sync_status(rt_scene* s) {
    if (!s) return RT_ERR_INVALID_ARG;
    rt_status st = rt_scene_sync_own(s);
    if (st != RT_OK && st != RT_ERR_CAPACITY) return st;
    bool ovf = st == RT_ERR_CAPACITY || s->split_dev_overflow;
    s->split_dev_overflow = false;
    if (s->split && s->split_dev_pending) {  // rt_render_frame_async's other share
        s->split_dev_pending = false;
        rt_status e = rt_multi_each(s->split, [&](rt_scene* c) -> rt_status {
            rt_status r = rt_scene_sync_own(c);
            if (r == RT_ERR_CAPACITY) {
                ovf = true;
                return RT_OK;
            }
            return r;
        });
        if (e != RT_OK) return e;
    }
    return ovf ? RT_ERR_CAPACITY : RT_OK;
}

rt_status rt_scene_sync_own(rt_scene* s) {
    if (!s) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(s->device));
    // every stream-ordered render of this handle is complete after this loop, so the events
    // are released (one per caller stream would otherwise accumulate for the process's life)
    for (auto& se : s->ev_streams) HIP_TRY(hipEventSynchronize(se.second));
    for (auto& se : s->ev_streams) (void)hipEventDestroy(se.second);
    s->ev_streams.clear();
    // an overflow a checked pass found latched before it rendered (rt_render_bands_ex_async)
    bool ovf = s->ovf_pending;
    s->ovf_pending = false;
    if (s->ws.overflow) {
        // read and clear the sticky word on the handle's own stream, waited for here: no
        // null-stream operation (unordered with the callers' non-blocking streams) touches it
        uint32_t v = 0;
        HIP_TRY(hipMemcpyAsync(&v, s->ws.overflow + 1, sizeof(v), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        if (v) {
            HIP_TRY(hipMemsetAsync(s->ws.overflow + 1, 0, sizeof(v), s->stream));
            HIP_TRY(hipStreamSynchronize(s->stream));
            ovf = true;
        }
    }
    if (!ovf) return RT_OK;
    // the next pass on this scene gets a pool twice as large (up to the index limit)
    s->pool_floor = (uint32_t)std::min<uint64_t>(2ull * s->ws.capacity, pool_cap_limit(s));
    return RT_ERR_CAPACITY;
}

rt_status rt_scene_clone(const rt_scene* src, int32_t device, rt_scene** out) {
    if (!src || !out) return RT_ERR_INVALID_ARG;
    std::unique_ptr<rt_scene> sc(new (std::nothrow) rt_scene());
    if (!sc) return RT_ERR_OUT_OF_MEMORY;
    rt_status st = select_device(device, &sc->device);
    if (st != RT_OK) return st;
    HIP_TRY(hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&sc->ev0));
    HIP_TRY(hipEventCreate(&sc->ev1));
    HIP_TRY(hipMalloc(&sc->dmem, src->dbytes));
    sc->dbytes = src->dbytes;
    // on the clone's own stream and waited for: a render on any caller stream sees the copy
    if (sc->device == src->device)
        HIP_TRY(hipMemcpyAsync(sc->dmem, src->dmem, src->dbytes, hipMemcpyDeviceToDevice, sc->stream));
    else
        HIP_TRY(hipMemcpyPeerAsync(sc->dmem, sc->device, src->dmem, src->device, src->dbytes, sc->stream));
    HIP_TRY(hipMemsetAsync((uint8_t*)sc->dmem + ((const uint8_t*)src->S.scan_ops - (const uint8_t*)src->dmem), 0,
                           RT_OPS_SLOTS * RT_OPS_STRIDE * sizeof(unsigned long long), sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    // the same DevScene, every pointer rebased into the new allocation
    sc->S = src->S;
    const uint8_t* from = (const uint8_t*)src->dmem;
    uint8_t* to = (uint8_t*)sc->dmem;
    auto rebase = [&](auto& ptr) {
        if (ptr) ptr = reinterpret_cast<std::remove_reference_t<decltype(ptr)>>(to + ((const uint8_t*)ptr - from));
    };
    DevScene& S = sc->S;
    rebase(S.dsph); rebase(S.gsph); rebase(S.tri); rebase(S.cube); rebase(S.plane); rebase(S.cubetri);
    rebase(S.shapes); rebase(S.mats); rebase(S.lights); rebase(S.bvh_nodes); rebase(S.bvh_leaves);
    rebase(S.graze_blk); rebase(S.graze_tri); rebase(S.graze_pn); rebase(S.graze_mask); rebase(S.scan_ops);
    sc->flops_per_scan = src->flops_per_scan;
    sc->normal_max = src->normal_max;
    sc->n_point_lights = src->n_point_lights;
    sc->num_cus = g_num_cus(sc->device);
    sc->count_ops = src->count_ops;
    sc->tune = src->tune;
    sc->d_mats = src->d_mats;
    sc->d_shapes = src->d_shapes;
    sc->d_lights = src->d_lights;
    sc->d_ambient = src->d_ambient;
    *out = sc.release();
    return RT_OK;
}

rt_status rt_unpermute_bands_async(const float* d_gathered, uint32_t x_res, uint32_t y_res,
                                   uint32_t band_rows, uint32_t world, float* d_frame, void* stream) {
    if (!d_gathered || !d_frame || band_rows == 0 || world == 0 || x_res == 0 || y_res == 0)
        return RT_ERR_INVALID_ARG;
    uint32_t rpr = rt_band_rows_per_rank(y_res, band_rows, world);
    HIP_TRY(launch_unpermute(d_gathered, x_res, y_res, band_rows, world, rpr, d_frame, (hipStream_t)stream));
    return RT_OK;
}

rt_status rt_unpermute_bands_u8_async(const uint8_t* d_gathered, uint32_t x_res, uint32_t y_res,
                                      uint32_t band_rows, uint32_t world, uint8_t* d_frame, void* stream) {
    if (!d_gathered || !d_frame || band_rows == 0 || world == 0 || x_res == 0 || y_res == 0)
        return RT_ERR_INVALID_ARG;
    uint32_t rpr = rt_band_rows_per_rank(y_res, band_rows, world);
    HIP_TRY(launch_unpermute_u8(d_gathered, x_res, y_res, band_rows, world, rpr, d_frame, (hipStream_t)stream));
    return RT_OK;
}

rt_status rt_unpermute_bands_batch_async(const float* d_gathered, uint32_t x_res, uint32_t y_res,
                                         uint32_t band_rows, uint32_t world, uint32_t n_frames,
                                         uint32_t stride_frames, float* d_frames, void* stream) {
    if (!d_gathered || !d_frames || band_rows == 0 || world == 0 || x_res == 0 || y_res == 0 || n_frames == 0 ||
        stride_frames < n_frames || n_frames > 65535u)
        return RT_ERR_INVALID_ARG;
    const uint32_t rpr = rt_band_rows_per_rank(y_res, band_rows, world);
    HIP_TRY(launch_unpermute(d_gathered, x_res, y_res, band_rows, world, rpr, d_frames, (hipStream_t)stream, n_frames,
                             stride_frames * rpr));
    return RT_OK;
}

rt_status rt_unpermute_bands_batch_u8_async(const uint8_t* d_gathered, uint32_t x_res, uint32_t y_res,
                                            uint32_t band_rows, uint32_t world, uint32_t n_frames,
                                            uint32_t stride_frames, uint8_t* d_frames, void* stream) {
    if (!d_gathered || !d_frames || band_rows == 0 || world == 0 || x_res == 0 || y_res == 0 || n_frames == 0 ||
        stride_frames < n_frames || n_frames > 65535u)
        return RT_ERR_INVALID_ARG;
    const uint32_t rpr = rt_band_rows_per_rank(y_res, band_rows, world);
    HIP_TRY(launch_unpermute_u8(d_gathered, x_res, y_res, band_rows, world, rpr, d_frames, (hipStream_t)stream,
                                n_frames, stride_frames * rpr));
    return RT_OK;
}

rt_status rt_quantize_u8_async(const float* d_rgb, size_t n, uint8_t* d_rgb8, void* stream) {
    if (!d_rgb || !d_rgb8) return RT_ERR_INVALID_ARG;
    if (n == 0) return RT_OK;
    HIP_TRY(launch_quantize(d_rgb, n, d_rgb8, (hipStream_t)stream));
    return RT_OK;
}

rt_status rt_render(const rt_scene* scene, const rt_camera* cam, uint32_t depth, const rt_render_opts* opts,
                    float* rgb, uint8_t* rgb8) {
    return rt_render_spp(scene, cam, depth, 1, 0, opts, rgb, rgb8);
}

rt_status rt_render_spp(const rt_scene* scene, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                        const rt_render_opts* opts, float* rgb, uint8_t* rgb8) {
    rt_scene* s = const_cast<rt_scene*>(scene);
    if (!s || !cam || !rgb || spp == 0) return RT_ERR_INVALID_ARG;
    if (opts && opts->device >= 0 && opts->device != s->device) return RT_ERR_INVALID_ARG;
    if (s->multi) return rt_multi_render(s, cam, depth, spp, seed, opts, rgb, rgb8);
    // One frame as S band shares of this device, rendered side by side on S streams (each
    // its own scene clone and workspace), exchanged by device copies and un-permuted: the
    // latency-bound tails of one share's levels overlap the other's work.  Tune::seam_split
    // (default 2; 1 = one pass), seam_band_rows (default: contiguous shares).  Config 3,
    // 1080p, one MI355X: 3.47 ms of device time against 4.09 for one pass (8-row bands: 3.69;
    // 3 shares: 3.80, 4: 5.08).
    const int split = s->tune.seam_split;
    if (split > 1 && cam->y_res >= 16u * (uint32_t)split) {
        if (s->split_dev_pending) {
            // a stream-ordered rt_render_frame_async on these shares is not reported yet: keep
            // its overflow for the caller's rt_scene_sync_status (this render's own status
            // checks below would otherwise consume it)
            rt_status ps = rt_scene_sync_status(s);
            if (ps == RT_ERR_CAPACITY)
                s->split_dev_overflow = true;
            else if (ps != RT_OK)
                return ps;
        }
        rt_status es = ensure_split(s, split);
        if (es != RT_OK) return es;
        // contiguous shares by default (top / bottom halves: 3.47 ms against 3.69 with 8-row
        // bands dealt in turn -- shares of different content fall out of step, so one share's
        // level tails meet the other's work)
        const uint32_t br = (uint32_t)s->tune.seam_band_rows;
        const uint32_t even = ((cam->y_res + (uint32_t)split - 1u) / (uint32_t)split + 7u) / 8u * 8u;
        // Two shares meet where share 1 finishes as share 0's rows reach the caller (share 0's
        // copy then runs under share 1's tail): after each render the row moves 8 rows toward
        // the share that is late on that mark (within [half, 3/4] of the frame: share 0 holds
        // one band only down to half the rows).  Config 3: share 0 (the top) is the cheaper
        // half; fixed rows 544 / 576 / 608 measured 3.38 / 3.35 / 3.37 ms of device time
        // (seam_band_rows pins the row, seam_adapt=0 keeps the even split, seam_adapt=device
        // balances the finish times alone)
        const bool adapt = !br && split == 2 && s->tune.seam_adapt != 0;
        const bool adapt_copy = s->tune.seam_adapt != 2;
        const uint32_t hi = std::max(even, (cam->y_res * 3u / 4u) / 8u * 8u);
        if (s->seam_y != cam->y_res || s->seam_rows < even || s->seam_rows > hi) {
            s->seam_rows = even;
            s->seam_y = cam->y_res;
            if (adapt && !s->tune.node_cap) {  // every share's node pool sized once for the largest
                                                // share it can get (unless the node_cap test knob
                                                // pins the pools)
                const uint64_t floor = std::min<uint64_t>((uint64_t)hi * cam->x_res * (uint64_t)s->tune.node_factor,
                                                          pool_cap_limit(s));
                auto raise = [&](rt_scene* c) {
                    c->pool_floor = std::max<uint32_t>(c->pool_floor, (uint32_t)floor);
                    return RT_OK;
                };
                (void)raise(s);
                (void)rt_multi_each(s->split, raise);
            }
        }
        const uint32_t rows = br ? br : (adapt ? s->seam_rows : even);
        rt_multi_set_band_rows(s->split, rows);
        // the shares' persistent grids at Tune::seam_grid_pct % of the chip (default 80: two
        // concurrent full-chip grids leave more blocks waiting for a slot; 100 / 90 / 80 at
        // the 576-row meeting: 3.35 / 3.31 - 3.34 / 3.30 - 3.31 ms), or the scene's own
        // share if that is smaller; restored afterwards
        const int pct = std::min(s->grid_pct, s->tune.seam_grid_pct);
        const int saved = s->grid_pct;
        auto set_pct = [&](int v) {
            s->grid_pct = v;
            (void)rt_multi_each(s->split, [&](rt_scene* c) {
                c->grid_pct = v;
                return RT_OK;
            });
        };
        set_pct(pct);
        rt_status st = rt_multi_render_state(s->split, cam, depth, spp, seed, opts, rgb, rgb8);
        set_pct(saved);
        if (st == RT_OK && adapt) {
            float t[2] = {0.f, 0.f}, c[2] = {0.f, 0.f};
            if (rt_multi_share_ms(s->split, t, 2) == RT_OK && t[0] > 0.f && t[1] > 0.f &&
                (!adapt_copy || rt_multi_copy_ms(s->split, c, 2) == RT_OK)) {
                // > 0: share 1 ends after share 0's rows are out -- share 0 can take more rows
                const float late = t[1] - (t[0] + c[0]), band = 0.03f * t[1];
                if (late > band && s->seam_rows + 8u <= hi)
                    s->seam_rows += 8u;
                else if (late < -band && s->seam_rows >= even + 8u)
                    s->seam_rows -= 8u;
            }
        }
        return st;
    }
    HIP_TRY(hipSetDevice(s->device));
    size_t n = (size_t)cam->x_res * cam->y_res * 3;
    // one band share holding every row: its buffer has the padded row count (the pass
    // zero-fills rows y_res .. rows_local - 1); the first y_res rows are the frame
    const size_t n_pad = (size_t)cam->x_res * rt_band_rows_per_rank(cam->y_res, 8, 1) * 3;
    rt_status st = ensure_ws(s, n_pad, rgb8 ? n_pad : 0);
    if (st != RT_OK) return st;
    hipStream_t stream = s->stream;
    for (int attempt = 0;; attempt++) {
        HIP_TRY(hipMemsetAsync(s->ws.counters, 0, 4 * sizeof(unsigned long long), stream));
        HIP_TRY(hipEventRecord(s->ev0, stream));
        // single device: one "band" holding every row; as_u8 fused into the level-0 combine
        const PassOut o{s->ws.out, rgb8 ? s->ws.out8 : nullptr, s->ws.counters, false, true};
        st = launch_bands(s, cam, depth, spp, seed, 8, 0, 1, o, stream);
        if (st != RT_OK) return st;
        HIP_TRY(hipEventRecord(s->ev1, stream));
        if (!s->ws.overflow) break;
        uint32_t ovf = 0;
        HIP_TRY(hipMemcpyAsync(&ovf, s->ws.overflow, sizeof(ovf), hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        if (!ovf) break;
        // node pool too small for this scene's ray trees: grow it and render again
        const uint64_t lim = pool_cap_limit(s);
        if (attempt >= 8 || s->ws.capacity >= lim) return RT_ERR_CAPACITY;
        rt_status g = grow_node_pool(s->ws, (uint32_t)std::min<uint64_t>(2ull * s->ws.capacity, lim));
        if (g != RT_OK) return g;
    }
    HIP_TRY(hipMemcpyAsync(rgb, s->ws.out, n * sizeof(float), hipMemcpyDeviceToHost, stream));
    if (rgb8) HIP_TRY(hipMemcpyAsync(rgb8, s->ws.out8, n, hipMemcpyDeviceToHost, stream));
    unsigned long long cnt[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(cnt, s->ws.counters, sizeof(cnt), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    if (opts && opts->counters) {
        opts->counters->node_rays = cnt[0];
        opts->counters->shadow_rays = cnt[1];
        opts->counters->pixels = cnt[2];
        opts->counters->wave_iterations = cnt[3];
    }
    if (opts && opts->kernel_ms) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        *opts->kernel_ms = ms;
    }
    return RT_OK;
}


// ---------------------------------------------------------------- ray forest
// render_tree.rs: generate_ray_forest (:147-164) keeps every intersection of every
// pixel's ray tree; render_forest (:121-127) shades the whole forest; render_forest_filter
// (:129-145) re-shades only trees that hold a mutated shape.  On the device the forest is
// the level-synchronous pipeline's node pool, kept after the trace + shadow passes, plus
// per node: material index, texture coordinates, `entering`, the shape id and the pixel.

}  // extern "C"

struct rt_forest {
    rt_scene* s = nullptr;
    uint64_t generation = 0;    // the scene's rt_scene::generation at creation
    rt_camera cam{};
    uint32_t depth = 0;
    Workspace ws;
    WaveParams p{};
    uint32_t levels[2 * (RT_MAX_DEPTH + 1) + 1] = {};  // (offset, count) per level, then levels used
    uint32_t n_nodes = 0;
    float* frame = nullptr;     // [y_res * x_res * 3] the last shade
    uint8_t* mark = nullptr;    // [pixels] dirty / tree-holds-id marks
    uint8_t* key_mask = nullptr;
    uint32_t n_keys = 0;
    uint32_t* sizes = nullptr;  // [pixels]
    unsigned long long* counters = nullptr;  // node, shadow, pixels of the build
    // device time of the build's last pass and of the last shade (rt_forest_timings)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    bool shaded = false;
};

namespace {

size_t forest_pixels(const rt_forest* f) { return (size_t)f->cam.x_res * f->cam.y_res; }

rt_status forest_shade(rt_forest* f, const uint8_t* dirty) {
    WaveParams p = f->p;
    p.S = f->s->S;  // current material table
    p.dirty = dirty;
    int cb = f->s->num_cus * (f->s->occ_combine > 0 ? f->s->occ_combine : 1);
    uint32_t used = f->levels[2 * (RT_MAX_DEPTH + 1)];
    for (uint32_t k = used; k-- > 0;) HIP_TRY(launch_forest_shade(p, k, cb, f->frame, f->s->stream));
    HIP_TRY(hipEventRecord(f->ev[3], f->s->stream));
    f->shaded = true;
    return RT_OK;
}
// a rebuild since the forest was made: its nodes' material indices and lit words describe
// the old scene, which the handle no longer holds (rt_api.h rt_scene_update)
bool forest_stale(const rt_forest* f) { return f->generation != f->s->generation; }

// mark[pixel] = tree holds one of `ids` (or sizes per pixel when ids == nullptr)
rt_status forest_mark(rt_forest* f, const int32_t* ids, uint32_t n_ids, bool sizes, hipEvent_t start = nullptr) {
    hipStream_t st = f->s->stream;
    size_t px = forest_pixels(f);
    const uint8_t* mask = nullptr;
    if (ids) {
        std::vector<uint8_t> h(f->n_keys, 0);
        for (uint32_t i = 0; i < n_ids; i++)
            if (ids[i] >= 0 && (uint32_t)ids[i] < f->n_keys) h[ids[i]] = 1;
        HIP_TRY(hipMemcpyAsync(f->key_mask, h.data(), f->n_keys, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemsetAsync(f->mark, 0, px, st));
        HIP_TRY(hipStreamSynchronize(st));  // h goes out of scope
        mask = f->key_mask;
    }
    if (sizes) HIP_TRY(hipMemsetAsync(f->sizes, 0, px * sizeof(uint32_t), st));
    if (start) HIP_TRY(hipEventRecord(start, st));
    HIP_TRY(launch_forest_mark(f->ws.node_key, f->ws.node_pixel, f->ws.node_flags, f->n_nodes, mask, f->n_keys, f->mark,
                               sizes ? f->sizes : nullptr, st));
    return RT_OK;
}

}  // namespace

extern "C" {

rt_status rt_forest_create(rt_scene* s, const rt_camera* cam, uint32_t depth, rt_forest** out) {
    if (!s || !cam || !out) return RT_ERR_INVALID_ARG;
    if (cam->x_res == 0 || cam->y_res == 0) return RT_ERR_INVALID_ARG;
    if (depth > RT_MAX_DEPTH) return RT_ERR_UNSUPPORTED;
    if ((uint64_t)cam->x_res * cam->y_res * 3 >= (1ull << 32)) return RT_ERR_UNSUPPORTED;
    HIP_TRY(hipSetDevice(s->device));
    std::unique_ptr<rt_forest> f(new (std::nothrow) rt_forest());
    if (!f) return RT_ERR_OUT_OF_MEMORY;
    f->s = s;
    f->generation = s->generation;
    f->cam = *cam;
    f->depth = depth;
    f->ws.forest = true;
    size_t px = forest_pixels(f.get());
    f->n_keys = std::max<uint32_t>((uint32_t)s->S.n_shapes, 12u);  // cube hits report ids 0..11
    struct Guard {  // frees everything if creation fails half way
        rt_forest* f;
        ~Guard() {
            if (!f) return;
            free_workspace(f->ws);
            for (void* b : {(void*)f->frame, (void*)f->mark, (void*)f->key_mask, (void*)f->sizes, (void*)f->counters})
                if (b) (void)hipFree(b);
            for (hipEvent_t e : f->ev)
                if (e) (void)hipEventDestroy(e);
        }
    } guard{f.get()};
    for (hipEvent_t& e : f->ev) HIP_TRY(hipEventCreate(&e));
    HIP_TRY(hipMalloc(&f->frame, px * 3 * sizeof(float)));
    HIP_TRY(hipMalloc(&f->mark, px));
    HIP_TRY(hipMalloc(&f->key_mask, f->n_keys));
    HIP_TRY(hipMalloc(&f->sizes, px * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&f->counters, 4 * sizeof(unsigned long long)));
    hipStream_t st = s->stream;
    const uint32_t band_rows = 8;
    for (int attempt = 0;; attempt++) {
        HIP_TRY(hipMemsetAsync(f->counters, 0, 4 * sizeof(unsigned long long), st));
        const PassOut o{nullptr, nullptr, f->counters, false, true};
        HIP_TRY(hipEventRecord(f->ev[0], st));
        rt_status r = wave_pipeline(s, f->ws, cam, depth, band_rows, 0, 1, o, st, &f->p, f->levels, 1, 0, 0, 1,
                                    nullptr, false, f->ev[1]);
        if (r != RT_OK) return r;
        uint32_t ovf = 0;
        HIP_TRY(hipMemcpyAsync(&ovf, f->ws.overflow, sizeof(ovf), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (!ovf) break;
        const uint64_t lim = pool_cap_limit(s);
        if (attempt >= 8 || f->ws.capacity >= lim) return RT_ERR_CAPACITY;
        rt_status g = grow_node_pool(f->ws, (uint32_t)std::min<uint64_t>(2ull * f->ws.capacity, lim));
        if (g != RT_OK) return g;
    }
    uint32_t used = f->levels[2 * (RT_MAX_DEPTH + 1)];
    f->n_nodes = used ? f->levels[2 * (used - 1)] + f->levels[2 * (used - 1) + 1] : 0;
    guard.f = nullptr;
    *out = f.release();
    return RT_OK;
}

rt_status rt_forest_destroy(rt_forest* f) {
    if (!f) return RT_ERR_INVALID_ARG;
    (void)hipSetDevice(f->s->device);
    (void)hipStreamSynchronize(f->s->stream);
    free_workspace(f->ws);
    for (void* b : {(void*)f->frame, (void*)f->mark, (void*)f->key_mask, (void*)f->sizes, (void*)f->counters})
        if (b) (void)hipFree(b);
    for (hipEvent_t e : f->ev)
        if (e) (void)hipEventDestroy(e);
    delete f;
    return RT_OK;
}

rt_status rt_forest_timings(const rt_forest* f, float* build_ms, float* shade_ms) {
    if (!f) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(f->s->device));
    if (build_ms) HIP_TRY(hipEventElapsedTime(build_ms, f->ev[0], f->ev[1]));
    if (shade_ms) {
        *shade_ms = 0.f;
        if (f->shaded) HIP_TRY(hipEventElapsedTime(shade_ms, f->ev[2], f->ev[3]));
    }
    return RT_OK;
}

rt_status rt_forest_render(rt_forest* f, float* rgb) {
    if (!f || !rgb) return RT_ERR_INVALID_ARG;
    if (forest_stale(f)) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(f->s->device));
    HIP_TRY(hipEventRecord(f->ev[2], f->s->stream));
    rt_status r = forest_shade(f, nullptr);
    if (r != RT_OK) return r;
    HIP_TRY(hipMemcpyAsync(rgb, f->frame, forest_pixels(f) * 3 * sizeof(float), hipMemcpyDeviceToHost,
                           f->s->stream));
    HIP_TRY(hipStreamSynchronize(f->s->stream));
    return RT_OK;
}

rt_status rt_forest_render_filter(rt_forest* f, const int32_t* mutated_ids, uint32_t n_ids, float* rgb) {
    if (!f || !rgb || (n_ids && !mutated_ids)) return RT_ERR_INVALID_ARG;
    if (forest_stale(f)) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(f->s->device));
    hipStream_t st = f->s->stream;
    size_t bytes = forest_pixels(f) * 3 * sizeof(float);
    HIP_TRY(hipMemcpyAsync(f->frame, rgb, bytes, hipMemcpyHostToDevice, st));  // untouched pixels keep these
    rt_status r = forest_mark(f, mutated_ids, n_ids, false, f->ev[2]);
    if (r != RT_OK) return r;
    r = forest_shade(f, f->mark);
    if (r != RT_OK) return r;
    HIP_TRY(hipMemcpyAsync(rgb, f->frame, bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return RT_OK;
}

rt_status rt_forest_tree_sizes(rt_forest* f, uint32_t* sizes) {
    if (!f || !sizes) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(f->s->device));
    rt_status r = forest_mark(f, nullptr, 0, true);
    if (r != RT_OK) return r;
    HIP_TRY(hipMemcpyAsync(sizes, f->sizes, forest_pixels(f) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           f->s->stream));
    HIP_TRY(hipStreamSynchronize(f->s->stream));
    return RT_OK;
}

rt_status rt_forest_trees_with(rt_forest* f, int32_t shape_id, uint64_t* count) {
    if (!f || !count) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(f->s->device));
    rt_status r = forest_mark(f, &shape_id, 1, false);
    if (r != RT_OK) return r;
    std::vector<uint8_t> m(forest_pixels(f));
    HIP_TRY(hipMemcpyAsync(m.data(), f->mark, m.size(), hipMemcpyDeviceToHost, f->s->stream));
    HIP_TRY(hipStreamSynchronize(f->s->stream));
    uint64_t n = 0;
    for (uint8_t v : m) n += v;
    *count = n;
    return RT_OK;
}

rt_status rt_forest_counters(const rt_forest* f, rt_counters* out) {
    if (!f || !out) return RT_ERR_INVALID_ARG;
    unsigned long long h[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpy(h, f->counters, sizeof(h), hipMemcpyDeviceToHost));
    out->node_rays = h[0];
    out->shadow_rays = h[1];
    out->pixels = h[2];
    out->wave_iterations = 0;
    return RT_OK;
}

rt_status rt_scene_set_material(rt_scene* s, uint32_t index, const rt_material* m) {
    if (!s || !m || index >= (uint32_t)s->S.n_mats) return RT_ERR_INVALID_ARG;
    MatRec cur;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    for (auto& se : s->ev_streams) HIP_TRY(hipEventSynchronize(se.second));  // renders on other streams
    HIP_TRY(hipMemcpyAsync(&cur, s->S.mats + index, sizeof(cur), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (m->kind != cur.kind) return RT_ERR_INVALID_ARG;  // the same kind, as the GUI's edits
    MatRec M;
    rt_status r = mat_rec(*m, M, s->normal_max);
    if (r != RT_OK) return r;
    // on the handle's stream, waited for: the next render on any caller stream sees the edit
    HIP_TRY(hipMemcpyAsync(const_cast<MatRec*>(s->S.mats) + index, &M, sizeof(M), hipMemcpyHostToDevice, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    // the handle's own copy is written first: rt_scene_update compares against it, so an edit
    // that reached this device must be recorded even if a band share or device below fails
    s->d_mats[index] = *m;
    if (s->split) {
        rt_status e = rt_multi_each(s->split, [&](rt_scene* c) { return rt_scene_set_material(c, index, m); });
        if (e != RT_OK) return e;
    }
    if (s->multi) {
        rt_status e = rt_multi_each(s->multi, [&](rt_scene* c) { return rt_scene_set_material(c, index, m); });
        if (e != RT_OK) return e;
    }
    return RT_OK;
}

rt_status rt_scene_update(rt_scene* s, const rt_scene_desc* d, int32_t* what) {
    if (what) *what = 0;
    if (!s || !d) return RT_ERR_INVALID_ARG;
    if ((d->n_materials && !d->materials) || (d->n_shapes && !d->shapes) || (d->n_lights && !d->lights))
        return RT_ERR_INVALID_ARG;
    auto same = [](const void* a, const void* b, size_t n) { return n == 0 || std::memcmp(a, b, n) == 0; };
    const bool geometry = d->n_shapes == s->d_shapes.size() && d->n_lights == s->d_lights.size() &&
                          d->n_materials == s->d_mats.size() &&
                          same(d->shapes, s->d_shapes.data(), d->n_shapes * sizeof(rt_shape)) &&
                          same(d->lights, s->d_lights.data(), d->n_lights * sizeof(rt_light)) &&
                          same(&d->ambient, &s->d_ambient, sizeof(rt_color));
    std::vector<uint32_t> edits;
    bool kinds = true;
    if (geometry) {
        for (uint32_t i = 0; i < d->n_materials; i++)
            if (!same(&d->materials[i], &s->d_mats[i], sizeof(rt_material))) {
                edits.push_back(i);
                kinds = kinds && d->materials[i].kind == s->d_mats[i].kind;
            }
        if (edits.empty()) return RT_OK;
    }
    // a stream-ordered render's unreported status is returned first (the update is then not
    // made), on every path that changes the scene
    rt_status st = rt_scene_sync_status(s);
    if (st != RT_OK) return st;
    if (s->multi) {
        st = rt_multi_each(s->multi, [](rt_scene* c) { return rt_scene_sync_status(c); });
        if (st != RT_OK) return st;
    }
    if (geometry && kinds) {
        // material edits of the same kind (the GUI's sliders, gui.rs:221-236) in place; every
        // edited material is validated before the first is applied (no partial update)
        for (uint32_t i : edits) {
            MatRec M;
            st = mat_rec(d->materials[i], M, s->normal_max);
            if (st != RT_OK) return st;
        }
        for (uint32_t i : edits) {
            st = rt_scene_set_material(s, i, &d->materials[i]);
            if (st != RT_OK) return st;
        }
        if (what) *what = 1;
        return RT_OK;
    }
    // anything else: the scene is rebuilt (same device and tuning) and adopted in place, so the
    // caller's handle, its stream, workspace and band shares stay valid
    rt_scene* fresh = nullptr;
    st = create_handle(d, s->device, s->tune, &fresh);
    if (st != RT_OK) return st;
    // every copy of the scene the handle renders with: its own, its band shares', its devices'
    std::vector<rt_scene*> targets{s};
    auto collect = [&](rt_scene* c) {
        targets.push_back(c);
        return RT_OK;
    };
    if (s->split) (void)rt_multi_each(s->split, collect);
    if (s->multi) (void)rt_multi_each(s->multi, collect);
    std::vector<void*> staged(targets.size(), nullptr);
    for (size_t i = 0; i < targets.size() && st == RT_OK; i++) st = stage_scene_data(targets[i], fresh, &staged[i]);
    if (st == RT_OK)
        for (size_t i = 0; i < targets.size(); i++) commit_scene_data(targets[i], fresh, staged[i]);
    else
        for (size_t i = 0; i < targets.size(); i++)
            if (staged[i]) {
                (void)hipSetDevice(targets[i]->device);
                (void)hipFree(staged[i]);
            }
    rt_scene_destroy(fresh);
    (void)hipSetDevice(s->device);
    if (st != RT_OK) return st;
    if (what) *what = 2;
    return RT_OK;
}

}  // extern "C"

#if RT_DIAG
// debug (tools/task_clock.py): copy the trace kernel's per wave-iteration records of the
// last RT_TASK_CLOCK render: out[0] = records written, then 4 words per record
extern "C" int rt_debug_task_clock(uint32_t* out, uint32_t max_records) {
    if (!g_task_clock) return 1;
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    return hipMemcpy(out, g_task_clock, (4 + 4 * (size_t)max_records) * sizeof(uint32_t), hipMemcpyDeviceToHost) ==
                   hipSuccess
               ? 0
               : 1;
}
#endif

// debug (tests/test_gpu_sort.py): the ray-queue radix sort on its own.  Sorts n device keys
// (their low `bits` bits) with digits of up to max_digit bits, stably; the values (d_vals, or
// the indices 0..n-1 when null) land in d_vals_out in key order.  Runs on the current device
// and synchronises it.
extern "C" int rt_debug_sort(const uint32_t* d_keys, const uint32_t* d_vals, uint32_t n, uint32_t bits,
                             uint32_t max_digit, uint32_t* d_vals_out) {
    if (!d_keys || !d_vals_out || bits == 0 || bits > 32) return RT_ERR_INVALID_ARG;
    if (n == 0) return RT_OK;
    uint32_t* levels = nullptr;
    uint32_t* tmp = nullptr;
    int rc = RT_OK;
    const size_t words = 4 * (size_t)n + (size_t)sort_max_digits() * sort_max_tiles(n) + sort_max_digits();
    if (hipMalloc(&levels, RT_LEVEL_TABLE_WORDS * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&tmp, words * sizeof(uint32_t)) != hipSuccess) {
        rc = RT_ERR_HIP;
    } else {
        // the shadow queue's slot: count at levels[2 (RT_MAX_DEPTH + 1)], offset 0
        std::vector<uint32_t> lv(RT_LEVEL_TABLE_WORDS, 0u);
        lv[2 * (RT_MAX_DEPTH + 1)] = n;
        uint32_t* tiles = tmp + 4 * (size_t)n;
        uint32_t* totals = tiles + (size_t)sort_max_digits() * sort_max_tiles(n);
        int cus = 0, dev = 0;
        if (hipMemcpy(levels, lv.data(), lv.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess ||
            hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            rc = RT_ERR_HIP;
        else if (launch_sort(levels, -1, n, bits, d_keys, d_vals, tmp, d_vals_out, tiles, totals, 4 * cus, 0,
                             max_digit) != hipSuccess ||
                 hipDeviceSynchronize() != hipSuccess)  // d_vals == null: the values are the indices
            rc = RT_ERR_HIP;
    }
    if (levels) (void)hipFree(levels);
    if (tmp) (void)hipFree(tmp);
    return rc;
}
