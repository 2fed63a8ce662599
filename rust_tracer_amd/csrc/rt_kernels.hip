// rt_kernels.hip -- the gfx950 megakernel for rust_tracer's render path.
//
// One persistent kernel owns the whole per-pixel work of src/render.rs:31-103:
// primary-ray generation (Camera::get_ray, render.rs:178-185), the linear nearest-hit
// scan (Scene::intersect, scene/mod.rs:98-116) over spheres / triangles / cubes /
// planes, the point-light shadow scans (PointLight::get_energy, mod.rs:189-206), Phong
// + Schlick shading (material.rs:77-93,165-213; render.rs:129-140) and the Whitted
// recursion (reflect_ray / refract_ray, render.rs:105-125).
//
// Execution model (MI355X-first, not a translation of the recursive CPU code):
//  * Each lane runs a small state machine whose every step is ONE scene scan: either the
//    nearest-hit scan of a tree node's ray or one shadow scan.  All lanes of a wave scan
//    the same primitive at the same time, so primitive records are wave-uniform and are
//    read with scalar (SMEM) loads; the per-lane work is pure f32 VALU.
//  * The recursion becomes a post-order continuation stack (frames in scratch, one per
//    pending tree level) so children combine into the parent exactly in the reference's
//    operation order: ((ambient + lights) + reflected) + refracted.
//  * Persistent workgroups; a lane that finishes its pixel takes the next one from a
//    global counter (wave-aggregated atomicAdd), so lanes stay busy while other lanes of
//    the wave are deep in a glass-sphere ray tree (lane-level compaction).
//
// Numerics: compiled with -ffp-contract=off, IEEE division/sqrt and f32 denormals on,
// so every +,-,*,/,sqrt is the same correctly rounded operation the reference
// executes, in the same order.  powf/atan2f/acosf come from ocml (<= 1-2 ulp from glibc).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_api.h"
#include "rt_device.hpp"

namespace rtdev {

#define RT_EPS 1.1920929e-07f  // std::f32::EPSILON

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mul(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// vector3.rs:91-94: three divisions by the length, not a reciprocal multiply
__device__ __forceinline__ V3 norm(V3 a) {
    float l = sqrtf(len2(a));
    return v3(a.x / l, a.y / l, a.z / l);
}
// matrix.rs:248-263 / 240-246 on rows r0..r2 = (m_i0, m_i1, m_i2, m_i3)
__device__ __forceinline__ V3 pt_mul(float4 r0, float4 r1, float4 r2, V3 p) {
    return v3(p.x * r0.x + p.y * r0.y + p.z * r0.z + r0.w, p.x * r1.x + p.y * r1.y + p.z * r1.z + r1.w,
              p.x * r2.x + p.y * r2.y + p.z * r2.z + r2.w);
}
__device__ __forceinline__ V3 vec3_mul(float4 r0, float4 r1, float4 r2, V3 v) {
    return v3(v.x * r0.x + v.y * r0.y + v.z * r0.z, v.x * r1.x + v.y * r1.y + v.z * r1.z,
              v.x * r2.x + v.y * r2.y + v.z * r2.z);
}
// inv_transform.transpose() * v  (sphere.rs:76, cube.rs:98)
__device__ __forceinline__ V3 tr_vec3_mul(float4 r0, float4 r1, float4 r2, V3 v) {
    return v3(v.x * r0.x + v.y * r1.x + v.z * r2.x, v.x * r0.y + v.y * r1.y + v.z * r2.y,
              v.x * r0.z + v.y * r1.z + v.z * r2.z);
}
__device__ __forceinline__ V3 xyz(float4 a) { return v3(a.x, a.y, a.z); }
__device__ __forceinline__ uint32_t keyof(float w) { return __float_as_uint(w); }

// Scene records are read through the constant address space: with wave-uniform indices
// the compiler then emits scalar (SMEM) loads into SGPRs, and every lane's VALU op takes
// the primitive's coefficients as a scalar operand.
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) float4 cfloat4;
#else
typedef const float4 cfloat4;  // host pass: the kernel body is never executed there
#endif
__device__ __forceinline__ cfloat4* cptr(const float4* p) { return (cfloat4*)p; }

// Nearest-hit bookkeeping: (t, key) lexicographic minimum == Scene::intersect's strict `<`
// in insertion order (ties keep the earlier shape / earlier cube triangle).
__device__ __forceinline__ void take(float t, uint32_t key, float& bt, uint32_t& bk) {
    bool better = (t < bt) | ((t == bt) & (key < bk));
    bt = better ? t : bt;
    bk = better ? key : bk;
}

// sphere.rs:126-145 + :66-77 on an object-space ray; returns t (false = no hit)
__device__ __forceinline__ bool sphere_t(V3 o, V3 d, float& t_out, bool& entering) {
    float a = len2(d);
    float b = 2.f * dot(d, o);  // l = o - Point3(0,0,0) == o
    float c = len2(o) - 1.f;
    float discr = b * b - 4.f * a * c;
    if (discr < 0.f) return false;
    float t0, t1;
    if (fabsf(discr) < RT_EPS) {
        float x = -0.5f * b / a;
        t0 = x;
        t1 = x;
    } else {
        float sq = sqrtf(discr);
        float q = (b > 0.f) ? -0.5f * (b + sq) : -0.5f * (b - sq);
        t0 = q / a;
        t1 = c / q;
    }
    if (t0 > t1) {
        float tmp = t1;
        t1 = t0;
        t0 = tmp;
    }
    if (t0 < 0.f && t1 < 0.f) return false;
    t_out = (t0 < 0.f) ? t1 : t0;
    entering = t0 > 0.f;
    return true;
}

// triangle.rs:51-80, Moller-Trumbore with e1 = v1 - v0, e2 = v2 - v0 precomputed
// (bit-identical: the host evaluates the same f32 subtractions).
// The division 1/det is only executed for lanes whose u-numerator can pass: for
// |det| <= 2^20 and a normal |un| the sign / magnitude pre-test below rejects exactly
// the lanes for which u = un * (1/det) would be < 0 or > 1.
__device__ __forceinline__ bool tri_hit(V3 o, V3 d, V3 v0, V3 e1, V3 e2, float& t_out,
                                        float& u_out, float& v_out, float& det_out) {
    V3 pvec = cross(d, e2);
    float det = dot(e1, pvec);
    if (fabsf(det) < RT_EPS) return false;
    V3 tvec = sub(o, v0);
    float un = dot(tvec, pvec);
    float adet = fabsf(det);
    bool opp = (un < 0.f) != (det < 0.f);
    bool early = (adet <= 1048576.f) &&
                 ((opp && (un != 0.f) && (fabsf(un) >= 1.17549435e-38f)) || (fabsf(un) > 2.f * adet));
    if (early) return false;
    float inv_det = 1.0f / det;
    float u = un * inv_det;
    if (u < 0.f || u > 1.f) return false;
    V3 qvec = cross(tvec, e1);
    float v = dot(d, qvec) * inv_det;
    if (v < 0.f || u + v > 1.f) return false;
    float t = dot(e2, qvec) * inv_det;
    if (t < 0.f) return false;
    t_out = t;
    u_out = u;
    v_out = v;
    det_out = det;
    return true;
}

// plane.rs:59-66: object-space ray, returns t (can be negative)
__device__ __forceinline__ bool plane_t(V3 o, V3 d, V3 n, V3 origin, float& t_out) {
    float denom = -dot(n, d);
    if (!(denom > RT_EPS)) return false;
    V3 dir = sub(origin, o);
    t_out = -dot(dir, n) / denom;
    return true;
}

// ------------------------------------------------------------------ the scan
// One pass over every primitive for one ray per lane.  All loop indices are
// wave-uniform, so records come in through the scalar cache.
__device__ __forceinline__ void scan(const DevScene& S, V3 o, V3 d, float& bt, uint32_t& bk) {
    bt = __builtin_huge_valf();
    bk = 0xFFFFFFFFu;
    // planes
    for (int i = 0; i < S.n_plane; ++i) {
        cfloat4* r = cptr(S.plane) + 5 * i;
        float4 r0 = r[0], r1 = r[1], r2 = r[2], rn = r[3], ro = r[4];
        V3 to = pt_mul(r0, r1, r2, o);
        V3 td = vec3_mul(r0, r1, r2, d);
        float t;
        if (plane_t(to, td, xyz(rn), xyz(ro), t)) take(t, keyof(rn.w), bt, bk);
    }
    // spheres with a translate*scale inverse: the zero off-diagonal products of pt_mul /
    // vec3_mul are skipped; x*m + (+-0) == x*m, so t is unchanged (only a zero's sign
    // can differ, which no comparison below observes).
    for (int i = 0; i < S.n_dsph; ++i) {
        cfloat4* r = cptr(S.dsph) + 2 * i;
        float4 s = r[0], off = r[1];
        V3 to = v3(o.x * s.x + off.x, o.y * s.y + off.y, o.z * s.z + off.z);
        V3 td = v3(d.x * s.x, d.y * s.y, d.z * s.z);
        float t;
        bool ent;
        if (sphere_t(to, td, t, ent)) take(t, keyof(s.w), bt, bk);
    }
    for (int i = 0; i < S.n_gsph; ++i) {
        cfloat4* r = cptr(S.gsph) + 4 * i;
        float4 r0 = r[0], r1 = r[1], r2 = r[2], rk = r[3];
        V3 to = pt_mul(r0, r1, r2, o);
        V3 td = vec3_mul(r0, r1, r2, d);
        float t;
        bool ent;
        if (sphere_t(to, td, t, ent)) take(t, keyof(rk.x), bt, bk);
    }
    for (int i = 0; i < S.n_tri; ++i) {
        cfloat4* r = cptr(S.tri) + 3 * i;
        float4 a = r[0], b = r[1], c = r[2];
        float t, u, v, det;
        if (tri_hit(o, d, xyz(a), xyz(b), xyz(c), t, u, v, det)) take(t, keyof(a.w), bt, bk);
    }
    for (int i = 0; i < S.n_cube; ++i) {
        cfloat4* r = cptr(S.cube) + 4 * i;
        float4 r0 = r[0], r1 = r[1], r2 = r[2], rk = r[3];
        V3 to = pt_mul(r0, r1, r2, o);
        V3 td = vec3_mul(r0, r1, r2, d);
        uint32_t key0 = keyof(rk.x);
#pragma unroll 2
        for (int k = 0; k < 12; ++k) {
            cfloat4* q = cptr(S.cubetri) + 4 * k;
            float t, u, v, det;
            if (tri_hit(to, td, xyz(q[0]), xyz(q[1]), xyz(q[2]), t, u, v, det))
                take(t, key0 | (uint32_t)k, bt, bk);
        }
    }
}

// ------------------------------------------------------------------ hit attributes
struct Hit {
    V3 p, n, eye;
    float tu, tv;
    float t;
    int32_t mat;
    bool entering;
};

__device__ __forceinline__ float4 ld4(const float* p) { return make_float4(p[0], p[1], p[2], p[3]); }

// Recompute the full Intersection of the chosen shape with the reference formulas
// (sphere.rs:57-98, plane.rs:59-84, triangle.rs:51-94, cube.rs:89-102).
__device__ Hit hit_attrs(const DevScene& S, uint32_t key, V3 o, V3 d, bool need_sphere_tex) {
    Hit h;
    const ShapeRec& R = S.shapes[key >> 4];
    h.mat = R.mat;
    float4 r0 = ld4(R.inv), r1 = ld4(R.inv + 4), r2 = ld4(R.inv + 8);
    h.eye = neg(norm(d));
    h.tu = 0.f;
    h.tv = 0.f;
    if (R.kind == RT_SHAPE_SPHERE) {
        V3 to = pt_mul(r0, r1, r2, o);
        V3 td = vec3_mul(r0, r1, r2, d);
        float t = 0.f;
        bool ent = false;
        sphere_t(to, td, t, ent);
        h.t = t;
        h.entering = ent;
        h.p = add(o, mul(d, t));
        V3 on = add(to, mul(td, t));
        V3 n = norm(tr_vec3_mul(r0, r1, r2, on));
        if (!ent) n = neg(n);
        h.n = n;
        if (need_sphere_tex) {  // sphere.rs:40-45
            const float PI_F = 3.14159265358979323846f;
            h.tu = (1.f + atan2f(n.z, n.x) / PI_F) * 0.5f;
            h.tv = acosf(n.y) / PI_F;
        }
    } else if (R.kind == RT_SHAPE_PLANE) {
        V3 to = pt_mul(r0, r1, r2, o);
        V3 td = vec3_mul(r0, r1, r2, d);
        V3 pn = v3(R.a[0], R.a[1], R.a[2]);
        V3 po = v3(R.a[3], R.a[4], R.a[5]);
        float t = 0.f;
        plane_t(to, td, pn, po, t);
        h.t = t;
        h.entering = t >= 0.f;
        h.p = add(o, mul(d, t));
        h.n = v3(R.a[6], R.a[7], R.a[8]);  // transform * normal, evaluated on the host
        h.tu = dot(v3(R.a[9], R.a[10], R.a[11]), h.p);
        h.tv = dot(v3(R.a[12], R.a[13], R.a[14]), h.p);
    } else if (R.kind == RT_SHAPE_TRIANGLE) {
        float t = 0.f, u = 0.f, v = 0.f, det = 0.f;
        tri_hit(o, d, v3(R.a[0], R.a[1], R.a[2]), v3(R.a[3], R.a[4], R.a[5]), v3(R.a[6], R.a[7], R.a[8]),
                t, u, v, det);
        h.t = t;
        h.p = add(o, mul(d, t));
        h.n = v3(R.a[9], R.a[10], R.a[11]);
        h.entering = det > 0.f;
        h.tu = u;
        h.tv = v;
    } else {  // cube
        V3 to = pt_mul(r0, r1, r2, o);
        V3 td = vec3_mul(r0, r1, r2, d);
        const float4* q = S.cubetri + 4 * (key & 15u);
        float t = 0.f, u = 0.f, v = 0.f, det = 0.f;
        tri_hit(to, td, xyz(q[0]), xyz(q[1]), xyz(q[2]), t, u, v, det);
        h.t = t;
        h.p = add(o, mul(d, t));
        h.n = norm(tr_vec3_mul(r0, r1, r2, xyz(q[3])));
        h.entering = det > 0.f;
        h.tu = u;
        h.tv = v;
    }
    return h;
}

// Saturating f32 -> i32 cast (Rust `as i32`: NaN -> 0)
__device__ __forceinline__ int32_t sat_i32(float x) {
    if (x != x) return 0;
    if (x >= 2147483648.f) return 2147483647;
    if (x <= -2147483648.f) return (int32_t)0x80000000u;
    return (int32_t)x;
}

// texture programs: CONST colour, or my_scene.rs:26-43 checkerboard
__device__ __forceinline__ V3 tex_eval(const TexRec& t, float tu, float tv) {
    if (t.kind == RT_TEX_CHECKERBOARD) {
        int32_t u = sat_i32(fabsf(tu));
        int32_t v = sat_i32(fabsf(tv));
        bool same = (tu < 0.f && tv < 0.f) || (tu > 0.f && tv > 0.f);
        bool white = same ? ((u % 2) == (v % 2)) : ((u % 2) != (v % 2));
        float c = white ? 1.f : 0.5f * 1.f;
        return v3(c, c, c);
    }
    return v3(t.r, t.g, t.b);
}

// render.rs:129-134; powi(5) = x * ((x*x)*(x*x)) (LLVM's square-and-multiply expansion)
__device__ __forceinline__ float fresnel_reflection(V3 l, V3 n, float n1, float n2) {
    float m_dot_r = dot(l, n);
    float q = (n1 - n2) / (n1 + n2);
    float r0 = q * q;
    float x = 1.f - m_dot_r;
    float x2 = x * x;
    float p5 = x * (x2 * x2);
    return r0 + (1.f - r0) * p5;
}

// Phong::get_reflected_energy (material.rs:77-93): lambert + phong, per channel
//   ((l.n * E) * Kd) + ((m.h ^ power * E) * Ks)   (phong term BLACK when m.h < 0)
__device__ __forceinline__ V3 reflected_energy(V3 E, V3 l, const Hit& h, V3 kd, V3 ks, float power) {
    float ln = dot(l, h.n);
    V3 hv = norm(add(norm(h.eye), norm(l)));
    float mh = dot(h.n, hv);
    V3 spec = v3(0.f, 0.f, 0.f);
    if (!(mh < 0.f)) {
        float pw = powf(mh, power);
        spec = v3((pw * E.x) * ks.x, (pw * E.y) * ks.y, (pw * E.z) * ks.z);
    }
    return v3((ln * E.x) * kd.x + spec.x, (ln * E.y) * kd.y + spec.y, (ln * E.z) * kd.z + spec.z);
}

// Continuation frame of a tree node whose children are still being traced.
struct Frame {
    float ax, ay, az;       // ambient + lights
    float fr, dr, pw, ft;   // reflected: fresnel, rdir.n, (m.h)^power; refracted: 1 - fresnel
    float kdx, kdy, kdz, ksx, ksy, ksz;
    float erx, ery, erz;    // colour returned by the reflection child
    float rox, roy, roz, rdx, rdy, rdz;  // pending refraction ray
    uint32_t flags;
};
enum : uint32_t {
    F_REFL = 1u,       // reflectivity > EPS: a reflected term exists
    F_SPEC = 2u,       // its phong part is not BLACK (m.h >= 0)
    F_REFR = 4u,       // refraction_index > EPS: a refracted term exists
    F_TIR = 8u,        // ... but refract_ray returned None
    F_WAIT_REFL = 16u, // waiting for the reflection child
    F_WAIT_REFR = 32u, // waiting for (or about to trace) the refraction child
    F_PEND_REFR = 64u  // refraction child still to be traced after the reflection child
};

// ((ambient + lights) + reflected) + refracted, render.rs:100
__device__ __forceinline__ V3 combine(const Frame& f, V3 er, V3 et) {
    V3 c = v3(f.ax, f.ay, f.az);
    if (f.flags & F_REFL) {
        V3 sp = v3(0.f, 0.f, 0.f);
        if (f.flags & F_SPEC) sp = v3((f.pw * er.x) * f.ksx, (f.pw * er.y) * f.ksy, (f.pw * er.z) * f.ksz);
        V3 d = v3((f.dr * er.x) * f.kdx + sp.x, (f.dr * er.y) * f.kdy + sp.y, (f.dr * er.z) * f.kdz + sp.z);
        c = add(c, v3(f.fr * d.x, f.fr * d.y, f.fr * d.z));
    } else {
        c = add(c, v3(0.f, 0.f, 0.f));
    }
    if (f.flags & F_REFR) {
        V3 inner = v3(0.f, 0.f, 0.f);
        if (!(f.flags & F_TIR)) inner = v3(f.ft * et.x, f.ft * et.y, f.ft * et.z);
        c = add(c, v3(f.kdx * inner.x, f.kdy * inner.y, f.kdz * inner.z));
    } else {
        c = add(c, v3(0.f, 0.f, 0.f));
    }
    return c;
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

template <int MAXF>
__global__ __launch_bounds__(256) void render_kernel(RenderParams P) {
    const DevScene& S = P.S;
    const V3 cam_o = v3(P.cam_ox, P.cam_oy, P.cam_oz);
    const uint32_t lane = lane_id();

    Frame st[MAXF > 0 ? MAXF : 1];

    // lane state
    int32_t item = -1;     // current work item (pixel), -1 = idle
    bool exhausted = false;
    uint32_t out_idx = 0;  // float index of this pixel in P.out
    V3 ro = v3(0, 0, 0), rd = v3(0, 0, 0);  // current node ray
    int32_t lvl = 0;       // tree level of the current node
    int32_t phase = 0;     // 0 = node scan, 1 = shadow scan for light `li`
    int32_t li = 0;
    unsigned long long n_node = 0, n_shadow = 0, n_pix = 0;

    // node being shaded
    Hit h;
    h.mat = 0;
    float n1 = 1.f, n2 = 1.f;
    V3 ka = v3(0, 0, 0), kd = v3(0, 0, 0), ks = v3(0, 0, 0), lsum = v3(0, 0, 0), ps = v3(0, 0, 0),
       ldir = v3(0, 0, 0);
    float power = 0.f;

    for (;;) {
        // ---- refill idle lanes with new pixels (one atomic per wave)
        for (;;) {
            uint64_t need = __ballot(item < 0 && !exhausted);
            if (need == 0) break;
            uint32_t first = (uint32_t)__builtin_ctzll(need);
            uint32_t cnt = (uint32_t)__builtin_popcountll(need);
            uint32_t base = 0;
            if (lane == first) base = atomicAdd(P.work_counter, cnt);
            base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)first);
            if (item < 0 && !exhausted) {
                uint32_t rank_in = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                uint32_t my = base + rank_in;
                if (my >= P.total_items) {
                    exhausted = true;
                } else {
                    uint32_t tile = my >> 6, w = my & 63u;
                    uint32_t u = (tile % P.tiles_x) * 8u + (w & 7u);
                    uint32_t lr = (tile / P.tiles_x) * 8u + (w >> 3);
                    uint32_t band = lr / P.band_rows;
                    uint32_t v = (band * P.world + P.rank) * P.band_rows + (lr - band * P.band_rows);
                    if (u < P.width && lr < P.rows_local && v < P.height) {
                        out_idx = (lr * P.width + u) * 3u;
                        n_pix++;
                        if (P.depth == 0) {  // trace_ray(.., 0) == BLACK
                            P.out[out_idx] = 0.f;
                            P.out[out_idx + 1] = 0.f;
                            P.out[out_idx + 2] = 0.f;
                        } else {
                            // Camera::get_ray (render.rs:178-185)
                            float x = P.x_min + (float)u * P.x_delta;
                            float y = P.y_max - (float)v * P.y_delta;
                            ro = cam_o;
                            rd = norm(sub(v3(x, y, 0.f), cam_o));
                            lvl = 0;
                            phase = 0;
                            item = (int32_t)my;
                        }
                    }
                }
            }
        }
        if (__ballot(item >= 0) == 0) break;
        if (item < 0) continue;

        // ---- one scene scan
        V3 so = (phase == 0) ? ro : ps;
        V3 sd = (phase == 0) ? rd : ldir;
        float bt;
        uint32_t bk;
        scan(S, so, sd, bt, bk);
        bool hit = bk != 0xFFFFFFFFu;

        bool node_done = false;
        bool returning = false;
        V3 ret = v3(0.f, 0.f, 0.f);

        if (phase == 0) {
            n_node++;
            if (!hit) {
                returning = true;  // trace_ray -> BLACK
            } else {
                const MatRec& M = S.mats[S.shapes[bk >> 4].mat];
                bool textured = M.kind == RT_MAT_TEXTURE_PHONG;
                h = hit_attrs(S, bk, ro, rd, textured);
                float ri = M.refraction_index;
                n1 = h.entering ? 1.f : ri;
                n2 = h.entering ? ri : 1.f;
                ka = tex_eval(M.ambient, h.tu, h.tv);
                kd = tex_eval(M.diffuse, h.tu, h.tv);
                ks = tex_eval(M.specular, h.tu, h.tv);
                power = M.power;
                lsum = v3(0.f, 0.f, 0.f);
                ps = add(h.p, mul(h.n, 0.0002f));  // render.rs:147
                li = 0;
                node_done = true;  // unless a point light needs a shadow scan (below)
            }
        } else {
            n_shadow++;
            const LightRec& L = S.lights[li];
            V3 lpos = v3(L.px, L.py, L.pz);
            bool shadowed = hit && (len2(sub(add(ps, mul(sd, bt)), ps)) < len2(sub(lpos, ps)));
            V3 E = shadowed ? v3(0.f, 0.f, 0.f) : v3(L.r, L.g, L.b);
            float f = fresnel_reflection(ldir, h.n, n1, n2);
            V3 g = reflected_energy(E, ldir, h, kd, ks, power);
            lsum = add(lsum, v3(f * g.x, f * g.y, f * g.z));
            li++;
            node_done = true;
        }

        if (node_done) {
            // advance over ambient lights (no scan) to the next point light
            bool need_scan = false;
            while (li < S.n_lights) {
                const LightRec& L = S.lights[li];
                if (L.kind == RT_LIGHT_POINT) {
                    ldir = norm(sub(v3(L.px, L.py, L.pz), ps));
                    phase = 1;
                    need_scan = true;
                    break;
                }
                V3 z = v3(0.f, 0.f, 0.f);
                float f = fresnel_reflection(z, h.n, n1, n2);
                V3 g = reflected_energy(v3(L.r, L.g, L.b), z, h, kd, ks, power);
                lsum = add(lsum, v3(f * g.x, f * g.y, f * g.z));
                li++;
            }
            if (need_scan) continue;

            // ---- the node is shaded: ambient + lights; set up its children
            const MatRec& M = S.mats[h.mat];
            Frame f;
            V3 amb = v3(ka.x * S.amb_r, ka.y * S.amb_g, ka.z * S.amb_b);
            V3 loc = add(amb, lsum);
            f.ax = loc.x; f.ay = loc.y; f.az = loc.z;
            f.kdx = kd.x; f.kdy = kd.y; f.kdz = kd.z;
            f.ksx = ks.x; f.ksy = ks.y; f.ksz = ks.z;
            f.erx = 0.f; f.ery = 0.f; f.erz = 0.f;
            f.fr = 0.f; f.dr = 0.f; f.pw = 0.f; f.ft = 0.f;
            f.rox = f.roy = f.roz = f.rdx = f.rdy = f.rdz = 0.f;
            f.flags = 0;
            bool child_ok = (uint32_t)(lvl + 1) < P.depth;
            V3 rro = v3(0, 0, 0), rrd = v3(0, 0, 0);
            bool trace_refl = false, trace_refr = false;
            if (M.reflectivity > RT_EPS) {  // render.rs:70-84 with reflect_ray :105-110
                f.flags |= F_REFL;
                V3 rv = sub(mul(h.n, 2.f * dot(rd, h.n)), rd);  // vector3.rs:113-115
                rrd = neg(norm(rv));
                rro = add(h.p, mul(rrd, 0.0002f));
                f.fr = fresnel_reflection(rrd, h.n, n1, n2);
                f.dr = dot(rrd, h.n);
                V3 hv = norm(add(norm(h.eye), norm(rrd)));
                float mh = dot(h.n, hv);
                if (!(mh < 0.f)) {
                    f.flags |= F_SPEC;
                    f.pw = powf(mh, power);
                }
                trace_refl = child_ok;
            }
            if (M.refraction_index > RT_EPS) {  // render.rs:86-98 with refract_ray :112-125
                f.flags |= F_REFR;
                float ratio = n1 / n2;
                float m_dot_r = -dot(rd, h.n);
                float cos2 = 1.f - ratio * ratio * (1.f - m_dot_r * m_dot_r);
                if (cos2 > 0.f) {
                    float ct = sqrtf(cos2);
                    V3 td = add(mul(rd, ratio), mul(h.n, ratio * m_dot_r - ct));
                    V3 to = add(h.p, mul(td, 0.0002f));
                    f.ft = 1.f - fresnel_reflection(td, neg(h.n), n1, n2);
                    f.rox = to.x; f.roy = to.y; f.roz = to.z;
                    f.rdx = td.x; f.rdy = td.y; f.rdz = td.z;
                    trace_refr = child_ok;
                } else {
                    f.flags |= F_TIR;
                }
            }
            if (!trace_refl && !trace_refr) {
                ret = combine(f, v3(0.f, 0.f, 0.f), v3(0.f, 0.f, 0.f));
                returning = true;
            } else {
                if (trace_refl) {
                    f.flags |= F_WAIT_REFL | (trace_refr ? F_PEND_REFR : 0u);
                    ro = rro;
                    rd = rrd;
                } else {
                    f.flags |= F_WAIT_REFR;
                    ro = v3(f.rox, f.roy, f.roz);
                    rd = v3(f.rdx, f.rdy, f.rdz);
                }
                st[lvl] = f;
                lvl++;
                phase = 0;
            }
        }

        if (returning) {
            // pop finished children into their parents (post-order)
            for (;;) {
                if (lvl == 0) {
                    P.out[out_idx] = ret.x;
                    P.out[out_idx + 1] = ret.y;
                    P.out[out_idx + 2] = ret.z;
                    item = -1;
                    break;
                }
                lvl--;
                Frame f = st[lvl];
                if (f.flags & F_WAIT_REFL) {
                    if (f.flags & F_PEND_REFR) {
                        st[lvl].erx = ret.x;
                        st[lvl].ery = ret.y;
                        st[lvl].erz = ret.z;
                        st[lvl].flags = (f.flags & ~(F_WAIT_REFL | F_PEND_REFR)) | F_WAIT_REFR;
                        ro = v3(f.rox, f.roy, f.roz);
                        rd = v3(f.rdx, f.rdy, f.rdz);
                        lvl++;
                        phase = 0;
                        break;
                    }
                    ret = combine(f, ret, v3(0.f, 0.f, 0.f));
                } else {
                    ret = combine(f, v3(f.erx, f.ery, f.erz), ret);
                }
            }
        }
    }

    // ---- counters: one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        n_node += __shfl_xor(n_node, off);
        n_shadow += __shfl_xor(n_shadow, off);
        n_pix += __shfl_xor(n_pix, off);
    }
    if (lane == 0 && P.ray_counters) {
        atomicAdd(P.ray_counters + 0, n_node);
        atomicAdd(P.ray_counters + 1, n_shadow);
        atomicAdd(P.ray_counters + 2, n_pix);
    }
}

// Scatter gathered per-rank band buffers into the row-major frame (one block row per frame row).
__global__ void unpermute_kernel(const float* __restrict__ in, uint32_t row_floats, uint32_t height,
                                 uint32_t band_rows, uint32_t world, uint32_t rows_per_rank,
                                 float* __restrict__ out) {
    uint32_t v = blockIdx.y;
    if (v >= height) return;
    uint32_t band = v / band_rows;
    uint32_t rank = band % world;
    uint32_t lr = (band / world) * band_rows + (v - band * band_rows);
    const float* src = in + ((size_t)rank * rows_per_rank + lr) * row_floats;
    float* dst = out + (size_t)v * row_floats;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < row_floats; i += gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// Color::as_u8 (color.rs:43-46): (255 * c) as u8, saturating, NaN -> 0
__global__ void quantize_kernel(const float* __restrict__ in, size_t n, uint8_t* __restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        float x = 255.f * in[i];
        uint8_t q = 0;
        if (x > 0.f) q = (x >= 255.f) ? (uint8_t)255 : (uint8_t)x;
        out[i] = q;
    }
}

}  // namespace rtdev

// ------------------------------------------------------------------ launch wrappers
namespace rtdev {

hipError_t launch_render(const RenderParams& p, int blocks, hipStream_t stream) {
    int maxf = (int)p.depth - 1;
    if (maxf <= 7) {
        hipLaunchKernelGGL(render_kernel<7>, dim3(blocks), dim3(256), 0, stream, p);
    } else if (maxf <= 15) {
        hipLaunchKernelGGL(render_kernel<15>, dim3(blocks), dim3(256), 0, stream, p);
    } else {
        hipLaunchKernelGGL(render_kernel<63>, dim3(blocks), dim3(256), 0, stream, p);
    }
    return hipGetLastError();
}

hipError_t render_occupancy(uint32_t depth, int* blocks_per_cu) {
    int maxf = (int)depth - 1;
    if (maxf <= 7) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, render_kernel<7>, 256, 0);
    if (maxf <= 15) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, render_kernel<15>, 256, 0);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, render_kernel<63>, 256, 0);
}

hipError_t launch_unpermute(const float* in, uint32_t x_res, uint32_t y_res, uint32_t band_rows,
                            uint32_t world, uint32_t rows_per_rank, float* out, hipStream_t stream) {
    uint32_t row_floats = x_res * 3u;
    dim3 grid((row_floats + 255) / 256, y_res);
    hipLaunchKernelGGL(unpermute_kernel, grid, dim3(256), 0, stream, in, row_floats, y_res, band_rows, world,
                       rows_per_rank, out);
    return hipGetLastError();
}

hipError_t launch_quantize(const float* in, size_t n, uint8_t* out, hipStream_t stream) {
    size_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(quantize_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, in, n, out);
    return hipGetLastError();
}

}  // namespace rtdev
