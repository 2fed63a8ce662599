// rt_api.cpp -- implementation of the C ABI (include/rt_api.h).
//
// Host side of the boundary: validate the flat scene description, run the scene-build
// preprocessing the reference performs in its constructors and set_transform calls
// (Matrix::inverse matrix.rs:99-153, Plane::new axes plane.rs:22-42, Triangle::new
// normal triangle.rs:16-39, Cube::new triangles cube.rs:21-77), lay the result out as
// the device runs of rt_device.hpp and upload it.  Rendering launches the megakernel of
// rt_kernels.hip; there is no CPU fallback anywhere in this library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_device.hpp"

namespace rtdev {
hipError_t launch_render(const RenderParams& p, int blocks, hipStream_t stream);
hipError_t render_occupancy(uint32_t depth, int* blocks_per_cu);
hipError_t launch_unpermute(const float* in, uint32_t x_res, uint32_t y_res, uint32_t band_rows,
                            uint32_t world, uint32_t rows_per_rank, float* out, hipStream_t stream);
hipError_t launch_quantize(const float* in, size_t n, uint8_t* out, hipStream_t stream);
bool rt_cube_table_check(const float* table);
hipError_t wave_occupancy(int* trace_blocks, int* shadow_blocks, int* combine_blocks);
hipError_t launch_wave_shadow(const WaveParams& p, int blocks, hipStream_t stream);
hipError_t launch_wave_init(uint32_t* levels, uint32_t n_words, uint32_t total_items, uint32_t* overflow,
                            hipStream_t stream);
hipError_t launch_wave_trace(const WaveParams& p, uint32_t level, int blocks, hipStream_t stream);
hipError_t launch_wave_combine(const WaveParams& p, uint32_t level, int blocks, hipStream_t stream);
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

struct Workspace {
    float* out = nullptr;            // device frame (rt_render)
    size_t out_floats = 0;
    uint8_t* out8 = nullptr;
    size_t out8_bytes = 0;
    unsigned long long* counters = nullptr;  // [node, shadow, pixels, wave iterations]
    uint32_t* work = nullptr;        // persistent-kernel work counter
    // level-synchronous pipeline
    Task* tasks = nullptr;
    NodeRec* nodes = nullptr;
    uint32_t capacity = 0;
    uint32_t* shadow = nullptr;      // shadow queue
    uint32_t shadow_capacity = 0;
    uint32_t* levels = nullptr;      // 2 * (RT_MAX_DEPTH + 2) words
    uint32_t* overflow = nullptr;
};

// Device path: "wave" (level-synchronous, default) or "mega" (per-pixel megakernel),
// chosen with RT_PIPELINE for A/B measurement.
bool use_megakernel() {
    const char* e = std::getenv("RT_PIPELINE");
    return e && std::strcmp(e, "mega") == 0;
}

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
    int occ[3] = {0, 0, 0};  // blocks per CU for the MAXF 7 / 15 / 63 variants
    int occ_trace = 0, occ_shadow = 0, occ_combine = 0;
    Workspace ws;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

namespace {

rt_status hip_status(hipError_t e) {
    if (e == hipSuccess) return RT_OK;
    if (e == hipErrorOutOfMemory) return RT_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return RT_ERR_NO_DEVICE;
    return RT_ERR_HIP;
}
#define HIP_TRY(x)                                  \
    do {                                            \
        hipError_t e_ = (x);                        \
        if (e_ != hipSuccess) return hip_status(e_); \
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

int variant_of(uint32_t depth) {
    int maxf = (int)depth - 1;
    return maxf <= 7 ? 0 : (maxf <= 15 ? 1 : 2);
}

rt_status ensure_ws(rt_scene* s, size_t out_floats, size_t out8_bytes) {
    Workspace& w = s->ws;
    if (!w.counters) {
        HIP_TRY(hipMalloc(&w.counters, 4 * sizeof(unsigned long long)));
        HIP_TRY(hipMalloc(&w.work, 64));
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

}  // namespace

extern "C" {

int32_t rt_api_version(void) { return RT_API_VERSION; }

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
    if (!d || !out) return RT_ERR_INVALID_ARG;
    if ((d->n_materials && !d->materials) || (d->n_shapes && !d->shapes) || (d->n_lights && !d->lights))
        return RT_ERR_INVALID_ARG;
    if (d->n_shapes >= (1u << 27)) return RT_ERR_UNSUPPORTED;

    // ---- host preprocessing into per-type runs
    std::vector<float> dsph, gsph, tri, cube, plane, cubetri;
    std::vector<ShapeRec> shapes(d->n_shapes);
    struct DiagSph {
        float s[3], o[3], key;
    };
    struct LooseTri {
        F3 v0, e1, e2;
        float key;
    };
    std::vector<DiagSph> diag_sph;
    std::vector<LooseTri> loose;
    uint64_t flops = 0;
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
            for (int c = 0; c < 4; c++) R.inv[r * 4 + c] = inv.m[r][c];
        float key = keyf(i << 4);
        switch (s.kind) {
            case RT_SHAPE_SPHERE: {
                bool diag = inv.m[0][1] == 0.f && inv.m[0][2] == 0.f && inv.m[1][0] == 0.f &&
                            inv.m[1][2] == 0.f && inv.m[2][0] == 0.f && inv.m[2][1] == 0.f;
                if (diag) {
                    diag_sph.push_back(DiagSph{{inv.m[0][0], inv.m[1][1], inv.m[2][2]},
                                           {inv.m[0][3], inv.m[1][3], inv.m[2][3]}, key});
                } else {
                    for (int r = 0; r < 3; r++) put4(gsph, inv.m[r][0], inv.m[r][1], inv.m[r][2], inv.m[r][3]);
                    put4(gsph, key, 0.f, 0.f, 0.f);
                }
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
                const float a[15] = {n.x, n.y, n.z, o.x, o.y, o.z, tn.x, tn.y, tn.z, u.x, u.y, u.z, v.x, v.y, v.z};
                std::memcpy(R.a, a, sizeof(a));
                for (int r = 0; r < 3; r++) put4(plane, inv.m[r][0], inv.m[r][1], inv.m[r][2], inv.m[r][3]);
                put4(plane, n.x, n.y, n.z, key);
                put4(plane, o.x, o.y, o.z, 0.f);
                flops += 49;
                break;
            }
            case RT_SHAPE_TRIANGLE: {
                F3 v0 = f3(s.data[0], s.data[1], s.data[2]);
                F3 v1 = f3(s.data[3], s.data[4], s.data[5]);
                F3 v2 = f3(s.data[6], s.data[7], s.data[8]);
                F3 e1 = fsub(v1, v0), e2 = fsub(v2, v0), nn = tri_normal(v0, v1, v2);
                const float a[12] = {v0.x, v0.y, v0.z, e1.x, e1.y, e1.z, e2.x, e2.y, e2.z, nn.x, nn.y, nn.z};
                std::memcpy(R.a, a, sizeof(a));
                loose.push_back(LooseTri{v0, e1, e2, key});
                flops += 52;
                break;
            }
            case RT_SHAPE_CUBE: {
                for (int r = 0; r < 3; r++) put4(cube, inv.m[r][0], inv.m[r][1], inv.m[r][2], inv.m[r][3]);
                put4(cube, key, 0.f, 0.f, 0.f);
                flops += 33 + 12 * 52;
                break;
            }
            default:
                return RT_ERR_INVALID_ARG;
        }
    }
    // diag spheres in pairs (2-wide packed scan); an odd one out joins the general run
    for (size_t k = 0; k + 1 < diag_sph.size(); k += 2) {
        const DiagSph &A = diag_sph[k], &B = diag_sph[k + 1];
        put4(dsph, A.s[0], B.s[0], A.s[1], B.s[1]);
        put4(dsph, A.s[2], B.s[2], A.o[0], B.o[0]);
        put4(dsph, A.o[1], B.o[1], A.o[2], B.o[2]);
        put4(dsph, A.key, B.key, 0.f, 0.f);
    }
    if (diag_sph.size() & 1) {
        const DiagSph& A = diag_sph.back();  // general form of the same inverse (exact formula)
        put4(gsph, A.s[0], 0.f, 0.f, A.o[0]);
        put4(gsph, 0.f, A.s[1], 0.f, A.o[1]);
        put4(gsph, 0.f, 0.f, A.s[2], A.o[2]);
        put4(gsph, A.key, 0.f, 0.f, 0.f);
    }
    // loose triangles in pairs; an odd count is padded with a degenerate triangle
    // (e1 = e2 = 0 -> det = 0 -> |det| < EPS: never a hit)
    if (loose.size() & 1) loose.push_back(LooseTri{f3(0, 0, 0), f3(0, 0, 0), f3(0, 0, 0), keyf(0xFFFFFFF0u)});
    for (size_t k = 0; k < loose.size(); k += 2) {
        const LooseTri &A = loose[k], &B = loose[k + 1];
        put4(tri, A.v0.x, B.v0.x, A.v0.y, B.v0.y);
        put4(tri, A.v0.z, B.v0.z, A.e1.x, B.e1.x);
        put4(tri, A.e1.y, B.e1.y, A.e1.z, B.e1.z);
        put4(tri, A.e2.x, B.e2.x, A.e2.y, B.e2.y);
        put4(tri, A.e2.z, B.e2.z, A.key, B.key);
        put4(tri, 0.f, 0.f, 0.f, 0.f);
    }
    cube_triangles(cubetri);
    if (!rt_cube_table_check(cubetri.data())) return RT_ERR_UNSUPPORTED;
    std::vector<MatRec> mats(d->n_materials);
    for (uint32_t i = 0; i < d->n_materials; i++) {
        const rt_material& m = d->materials[i];
        if (m.kind != RT_MAT_PHONG && m.kind != RT_MAT_TEXTURE_PHONG) return RT_ERR_INVALID_ARG;
        const rt_texture* tx[3] = {&m.ambient, &m.diffuse, &m.specular};
        for (int k = 0; k < 3; k++) {
            if (tx[k]->kind != RT_TEX_CONST && tx[k]->kind != RT_TEX_CHECKERBOARD) return RT_ERR_INVALID_ARG;
            // Phong ignores texture programs: its colours are constants (material.rs:55-65)
            if (m.kind == RT_MAT_PHONG && tx[k]->kind != RT_TEX_CONST) return RT_ERR_INVALID_ARG;
        }
        MatRec& M = mats[i];
        std::memset(&M, 0, sizeof(M));
        M.kind = m.kind;
        M.power = m.power;
        M.reflectivity = m.reflectivity;
        M.refraction_index = m.refraction_index;
        M.ambient = TexRec{m.ambient.kind, m.ambient.color.r, m.ambient.color.g, m.ambient.color.b};
        M.diffuse = TexRec{m.diffuse.kind, m.diffuse.color.r, m.diffuse.color.g, m.diffuse.color.b};
        M.specular = TexRec{m.specular.kind, m.specular.color.r, m.specular.color.g, m.specular.color.b};
    }
    if (d->n_lights > 32) return RT_ERR_UNSUPPORTED;  // shadow results are a 32-bit mask per node
    uint32_t n_point = 0;
    std::vector<LightRec> lights(d->n_lights);
    for (uint32_t i = 0; i < d->n_lights; i++) {
        const rt_light& l = d->lights[i];
        if (l.kind != RT_LIGHT_POINT && l.kind != RT_LIGHT_AMBIENT) return RT_ERR_INVALID_ARG;
        lights[i] = LightRec{l.kind, l.pos[0], l.pos[1], l.pos[2], l.color.r, l.color.g, l.color.b, 0.f};
        if (l.kind == RT_LIGHT_POINT) n_point++;
    }

    // ---- one allocation, 256-B aligned sections
    struct Sec {
        const void* src;
        size_t bytes;
        size_t off;
    };
    Sec secs[9] = {{dsph.data(), dsph.size() * 4, 0},       {gsph.data(), gsph.size() * 4, 0},
                   {tri.data(), tri.size() * 4, 0},         {cube.data(), cube.size() * 4, 0},
                   {plane.data(), plane.size() * 4, 0},     {cubetri.data(), cubetri.size() * 4, 0},
                   {shapes.data(), shapes.size() * sizeof(ShapeRec), 0},
                   {mats.data(), mats.size() * sizeof(MatRec), 0},
                   {lights.data(), lights.size() * sizeof(LightRec), 0}};
    size_t total = 0;
    for (auto& s : secs) {
        s.off = total;
        total += (s.bytes + 96 + 255) & ~(size_t)255;  // + one record group of look-ahead slack
    }
    if (total == 0) total = 256;

    std::unique_ptr<rt_scene> sc(new (std::nothrow) rt_scene());
    if (!sc) return RT_ERR_OUT_OF_MEMORY;
    rt_status st = select_device(device, &sc->device);
    if (st != RT_OK) return st;
    HIP_TRY(hipMalloc(&sc->dmem, total));
    sc->dbytes = total;
    std::vector<uint8_t> host(total, 0);
    for (auto& s : secs)
        if (s.bytes) std::memcpy(host.data() + s.off, s.src, s.bytes);
    HIP_TRY(hipMemcpy(sc->dmem, host.data(), total, hipMemcpyHostToDevice));
    auto at = [&](int k) { return (const void*)((const uint8_t*)sc->dmem + secs[k].off); };
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
    S.n_dsph = (int32_t)(dsph.size() / 16);  // pairs
    S.n_gsph = (int32_t)(gsph.size() / 16);
    S.n_tri = (int32_t)(tri.size() / 24);    // pairs
    S.n_cube = (int32_t)(cube.size() / 16);
    S.n_plane = (int32_t)(plane.size() / 20);
    S.n_shapes = (int32_t)d->n_shapes;
    S.n_lights = (int32_t)d->n_lights;
    S.n_mats = (int32_t)d->n_materials;
    S.amb_r = d->ambient.r;
    S.amb_g = d->ambient.g;
    S.amb_b = d->ambient.b;
    sc->flops_per_scan = flops;
    sc->n_point_lights = n_point;
    sc->num_cus = g_num_cus(sc->device);
    HIP_TRY(hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&sc->ev0));
    HIP_TRY(hipEventCreate(&sc->ev1));
    *out = sc.release();
    return RT_OK;
}

rt_status rt_scene_destroy(rt_scene* s) {
    if (!s) return RT_ERR_INVALID_ARG;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->ws.out) (void)hipFree(s->ws.out);
    if (s->ws.out8) (void)hipFree(s->ws.out8);
    if (s->ws.counters) (void)hipFree(s->ws.counters);
    if (s->ws.work) (void)hipFree(s->ws.work);
    if (s->ws.tasks) (void)hipFree(s->ws.tasks);
    if (s->ws.shadow) (void)hipFree(s->ws.shadow);
    if (s->ws.nodes) (void)hipFree(s->ws.nodes);
    if (s->ws.levels) (void)hipFree(s->ws.levels);
    if (s->ws.overflow) (void)hipFree(s->ws.overflow);
    if (s->dmem) (void)hipFree(s->dmem);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return RT_OK;
}

uint64_t rt_scene_flops_per_scan(const rt_scene* s) { return s ? s->flops_per_scan : 0; }
uint64_t rt_scene_device_bytes(const rt_scene* s) { return s ? (uint64_t)s->dbytes : 0; }

static rt_status launch_bands_wave(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t band_rows,
                                   uint32_t rank, uint32_t world, float* d_rgb, unsigned long long* d_counters,
                                   hipStream_t stream);

static rt_status launch_bands(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t band_rows,
                              uint32_t rank, uint32_t world, float* d_rgb, unsigned long long* d_counters,
                              hipStream_t stream) {
    if (!s || !cam || !d_rgb || band_rows == 0 || world == 0 || rank >= world) return RT_ERR_INVALID_ARG;
    if (cam->x_res == 0 || cam->y_res == 0) return RT_ERR_INVALID_ARG;
    if (depth > RT_MAX_DEPTH) return RT_ERR_UNSUPPORTED;
    if ((uint64_t)cam->x_res * cam->y_res * 3 >= (1ull << 32)) return RT_ERR_UNSUPPORTED;
    rt_status st = ensure_ws(s, 0, 0);
    if (st != RT_OK) return st;
    if (!use_megakernel())
        return launch_bands_wave(s, cam, depth, band_rows, rank, world, d_rgb, d_counters, stream);
    RenderParams p;
    std::memset(&p, 0, sizeof(p));
    p.S = s->S;
    p.cam_ox = cam->origin[0];
    p.cam_oy = cam->origin[1];
    p.cam_oz = cam->origin[2];
    p.x_min = cam->x_min;
    p.y_max = cam->y_max;
    // render.rs:179-180, evaluated once in f32 (identical on host and device)
    p.x_delta = (cam->x_max - cam->x_min) / (float)cam->x_res;
    p.y_delta = (cam->y_max - cam->y_min) / (float)cam->y_res;
    p.width = cam->x_res;
    p.height = cam->y_res;
    p.depth = depth;
    p.band_rows = band_rows;
    p.rank = rank;
    p.world = world;
    p.rows_local = rt_band_rows_per_rank(cam->y_res, band_rows, world);
    p.tiles_x = (cam->x_res + 7) / 8;
    uint32_t tiles_y = (p.rows_local + 7) / 8;
    p.total_items = p.tiles_x * tiles_y * 64u;
    p.out = d_rgb;
    p.ray_counters = d_counters;
    p.iter_counter = s->ws.counters + 3;
    p.work_counter = s->ws.work;

    int var = variant_of(depth);
    if (s->occ[var] == 0) {
        int b = 0;
        HIP_TRY(render_occupancy(depth, &b));
        s->occ[var] = b > 0 ? b : 1;
    }
    long long blocks = (long long)s->num_cus * s->occ[var];
    long long need = ((long long)p.total_items + 255) / 256;
    if (blocks > need) blocks = need;
    if (blocks < 1) blocks = 1;
    HIP_TRY(hipMemsetAsync(s->ws.work, 0, sizeof(uint32_t), stream));
    HIP_TRY(launch_render(p, (int)blocks, stream));
    return RT_OK;
}

// Level-synchronous pipeline: trace(0..L-1), then combine(L-1..0), all on `stream`.
static rt_status launch_bands_wave(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t band_rows,
                                   uint32_t rank, uint32_t world, float* d_rgb, unsigned long long* d_counters,
                                   hipStream_t stream) {
    WaveParams p;
    std::memset(&p, 0, sizeof(p));
    p.S = s->S;
    p.cam_ox = cam->origin[0];
    p.cam_oy = cam->origin[1];
    p.cam_oz = cam->origin[2];
    p.x_min = cam->x_min;
    p.y_max = cam->y_max;
    p.x_delta = (cam->x_max - cam->x_min) / (float)cam->x_res;  // render.rs:179-180
    p.y_delta = (cam->y_max - cam->y_min) / (float)cam->y_res;
    p.width = cam->x_res;
    p.height = cam->y_res;
    p.depth = depth;
    p.band_rows = band_rows;
    p.rank = rank;
    p.world = world;
    p.rows_local = rt_band_rows_per_rank(cam->y_res, band_rows, world);
    p.tiles_x = (cam->x_res + 7) / 8;
    uint64_t total = (uint64_t)p.tiles_x * ((p.rows_local + 7) / 8) * 64u;
    if (total >= (1ull << 30)) return RT_ERR_UNSUPPORTED;
    p.total_items = (uint32_t)total;
    // node / task pool: level 0 plus room for ~11 secondary nodes per pixel on average
    // (config 3 needs 2.7); an overflow is reported, never silently truncated
    uint64_t want = std::max<uint64_t>(total * 12u, 1u << 20);
    if (want > 0x7FFFFFFFu) want = 0x7FFFFFFFu;
    Workspace& w = s->ws;
    if (w.capacity < want) {  // grows only (rt_render may have grown it after an overflow)
        if (w.tasks) (void)hipFree(w.tasks);
        if (w.nodes) (void)hipFree(w.nodes);
        w.tasks = nullptr;
        w.nodes = nullptr;
        w.capacity = 0;
        HIP_TRY(hipMalloc(&w.tasks, want * sizeof(Task)));
        HIP_TRY(hipMalloc(&w.nodes, want * sizeof(NodeRec)));
        w.capacity = (uint32_t)want;
    }
    if (!w.levels) {
        HIP_TRY(hipMalloc(&w.levels, 2 * (RT_MAX_DEPTH + 2) * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&w.overflow, 64));
    }
    // shadow queue: one entry per point light per hit node
    uint64_t want_sh = std::min<uint64_t>((uint64_t)w.capacity * s->n_point_lights, 0x7FFFFFFFu);
    if (want_sh == 0) want_sh = 1;
    if (w.shadow_capacity < want_sh) {
        if (w.shadow) (void)hipFree(w.shadow);
        w.shadow = nullptr;
        w.shadow_capacity = 0;
        HIP_TRY(hipMalloc(&w.shadow, want_sh * sizeof(uint32_t)));
        w.shadow_capacity = (uint32_t)want_sh;
    }
    p.capacity = w.capacity;
    p.shadow_capacity = w.shadow_capacity;
    p.shadow = w.shadow;
    p.tasks = w.tasks;
    p.nodes = w.nodes;
    p.levels = w.levels;
    p.overflow = w.overflow;
    p.out = d_rgb;
    p.ray_counters = d_counters;
    if (s->occ_trace == 0) {
        int a = 0, b = 0, c = 0;
        HIP_TRY(wave_occupancy(&a, &b, &c));
        s->occ_trace = a > 0 ? a : 1;
        s->occ_shadow = b > 0 ? b : 1;
        s->occ_combine = c > 0 ? c : 1;
    }
    int tb = s->num_cus * s->occ_trace;
    int sb = s->num_cus * s->occ_shadow;
    int cb = s->num_cus * s->occ_combine;
    uint32_t levels = depth > 0 ? depth : 1;
    HIP_TRY(launch_wave_init(w.levels, 2 * (RT_MAX_DEPTH + 2), p.total_items, w.overflow, stream));
    for (uint32_t k = 0; k < levels; k++) HIP_TRY(launch_wave_trace(p, k, tb, stream));
    HIP_TRY(launch_wave_shadow(p, sb, stream));
    for (uint32_t k = levels; k-- > 0;) HIP_TRY(launch_wave_combine(p, k, cb, stream));
    return RT_OK;
}

rt_status rt_render_bands_async(const rt_scene* scene, const rt_camera* cam, uint32_t depth,
                                uint32_t band_rows, uint32_t rank, uint32_t world, float* d_rgb,
                                uint64_t* d_counters, void* stream) {
    rt_scene* s = const_cast<rt_scene*>(scene);
    if (!s) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(s->device));
    return launch_bands(s, cam, depth, band_rows, rank, world, d_rgb,
                        reinterpret_cast<unsigned long long*>(d_counters), (hipStream_t)stream);
}

rt_status rt_unpermute_bands_async(const float* d_gathered, uint32_t x_res, uint32_t y_res,
                                   uint32_t band_rows, uint32_t world, float* d_frame, void* stream) {
    if (!d_gathered || !d_frame || band_rows == 0 || world == 0 || x_res == 0 || y_res == 0)
        return RT_ERR_INVALID_ARG;
    uint32_t rpr = rt_band_rows_per_rank(y_res, band_rows, world);
    HIP_TRY(launch_unpermute(d_gathered, x_res, y_res, band_rows, world, rpr, d_frame, (hipStream_t)stream));
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
    rt_scene* s = const_cast<rt_scene*>(scene);
    if (!s || !cam || !rgb) return RT_ERR_INVALID_ARG;
    if (opts && opts->device >= 0 && opts->device != s->device) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(s->device));
    size_t n = (size_t)cam->x_res * cam->y_res * 3;
    rt_status st = ensure_ws(s, n, rgb8 ? n : 0);
    if (st != RT_OK) return st;
    hipStream_t stream = s->stream;
    for (int attempt = 0;; attempt++) {
        HIP_TRY(hipMemsetAsync(s->ws.counters, 0, 4 * sizeof(unsigned long long), stream));
        HIP_TRY(hipEventRecord(s->ev0, stream));
        // single device: one "band" holding every row
        st = launch_bands(s, cam, depth, 8, 0, 1, s->ws.out, s->ws.counters, stream);
        if (st != RT_OK) return st;
        HIP_TRY(hipEventRecord(s->ev1, stream));
        if (use_megakernel() || !s->ws.overflow) break;
        uint32_t ovf = 0;
        HIP_TRY(hipMemcpyAsync(&ovf, s->ws.overflow, sizeof(ovf), hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        if (!ovf) break;
        // node pool too small for this scene's ray trees: grow it and render again
        if (attempt >= 6 || s->ws.capacity >= 0x40000000u) return RT_ERR_OUT_OF_MEMORY;
        uint32_t cap = s->ws.capacity * 2u;
        (void)hipFree(s->ws.tasks);
        (void)hipFree(s->ws.nodes);
        s->ws.tasks = nullptr;
        s->ws.nodes = nullptr;
        s->ws.capacity = 0;
        HIP_TRY(hipMalloc(&s->ws.tasks, (size_t)cap * sizeof(Task)));
        HIP_TRY(hipMalloc(&s->ws.nodes, (size_t)cap * sizeof(NodeRec)));
        s->ws.capacity = cap;
    }
    if (rgb8) HIP_TRY(launch_quantize(s->ws.out, n, s->ws.out8, stream));
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

}  // extern "C"
