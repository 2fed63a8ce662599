// rt_common.hpp -- device code shared by the render kernels: f32 vector helpers in the
// reference's operation order, the nearest-hit scan (rt_scan.hpp), hit attributes of
// the chosen shape, texture programs, Schlick/Phong shading and the post-order combine.
//
// Numerics: compiled with -ffp-contract=off, IEEE division/sqrt and f32 denormals on,
// so every +,-,*,/,sqrt is the same correctly rounded operation the reference
// executes, in the same order.  powf, atan2f and acosf are glibc's own evaluations
// (rt_powf.hpp, rt_libmf.hpp: bit-identical to the reference's libm).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_api.h"
#include "rt_device.hpp"
#include "rt_libmf.hpp"
#include "rt_powf.hpp"
// the specular power (material.rs:211): glibc's powf, bit for bit (rt_powf.hpp); its tables in
// LDS (+1% over constant-memory reads): every kernel that shades calls rt_pow_stage() first
__shared__ rtpow::Log2Entry rt_pow_log2[16];
__shared__ uint64_t rt_pow_exp2[32];
struct LdsTabs {
    __device__ static inline rtpow::Log2Entry log2(int i) { return rt_pow_log2[i]; }
    __device__ static inline uint64_t exp2(uint32_t i) { return rt_pow_exp2[i]; }
};
__device__ __forceinline__ void rt_pow_stage() {
    if (threadIdx.x < 16) rt_pow_log2[threadIdx.x] = rtpow::kLog2Tab[threadIdx.x];
    if (threadIdx.x < 32) rt_pow_exp2[threadIdx.x] = rtpow::kExp2Tab[threadIdx.x];
    __syncthreads();
}
#define RT_POW(x, y) rtpow::powf_glibc<true, LdsTabs>((x), (y))

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
// A light record (wave-uniform index): two scalar loads.  Read through a generic pointer the
// loop over the lights became a chain of vector loads, each waited for with vmcnt(0) -- after
// every store the wave had outstanding.
__device__ __forceinline__ LightRec light_at(const DevScene& S, int i) {
    static_assert(sizeof(LightRec) == 32, "LightRec is two float4");
    cfloat4* p = cptr(reinterpret_cast<const float4*>(S.lights)) + 2 * i;
    const float4 a = p[0], b = p[1];
    LightRec L;
    L.kind = __float_as_int(a.x);
    L.px = a.y;
    L.py = a.z;
    L.pz = a.w;
    L.r = b.x;
    L.g = b.y;
    L.b = b.z;
    L.lb_base = __float_as_uint(b.w);
    return L;
}

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

#include "rt_scan.hpp"

// ------------------------------------------------------------------ hit attributes
struct Hit {
    V3 p, n, eye;
    float tu, tv;
    float t;
    int32_t mat;
    bool entering;
};

__device__ __forceinline__ float4 ld4(const float* p) { return make_float4(p[0], p[1], p[2], p[3]); }

// Shape and material records read whole, every 16-B piece requested at once: read field by
// field through a reference, the per-kind branches split the loads into dependent round
// trips (several L2 latencies per hit).
struct ShapeW {
    float4 w[8];  // {kind, mat, centre key, pad1} {inv row 0} {inv row 1} {inv row 2} {a[0..15]}
    __device__ __forceinline__ int32_t kind() const { return __float_as_int(w[0].x); }
    __device__ __forceinline__ int32_t mat() const { return __float_as_int(w[0].y); }
    __device__ __forceinline__ float a(int i) const {
        const float4 q = w[4 + (i >> 2)];
        const int c = i & 3;
        return c == 0 ? q.x : (c == 1 ? q.y : (c == 2 ? q.z : q.w));
    }
};
__device__ __forceinline__ ShapeW load_shape(const ShapeRec* shapes, uint32_t i) {
    static_assert(sizeof(ShapeRec) == 128, "ShapeRec is eight float4");
    const float4* p = reinterpret_cast<const float4*>(shapes + i);
    ShapeW r;
#pragma unroll
    for (int k = 0; k < 8; k++) r.w[k] = p[k];
    return r;
}
__device__ __forceinline__ MatRec load_mat(const MatRec* mats, uint32_t i) {
    static_assert(sizeof(MatRec) == 80, "MatRec is five float4");
    const float4* p = reinterpret_cast<const float4*>(mats + i);
    const float4 a = p[0], b = p[1], c = p[2], d = p[3], e = p[4];
    MatRec M;
    M.kind = __float_as_int(a.x);
    M.dark_zero = __float_as_int(a.y);
    M.power = a.z;
    M.reflectivity = a.w;
    M.refraction_index = b.x;
    M.pad1 = b.y;
    M.pad2 = b.z;
    M.pad3 = b.w;
    M.ambient = TexRec{__float_as_int(c.x), c.y, c.z, c.w};
    M.diffuse = TexRec{__float_as_int(d.x), d.y, d.z, d.w};
    M.specular = TexRec{__float_as_int(e.x), e.y, e.z, e.w};
    return M;
}

// Recompute the full Intersection of the chosen shape with the reference formulas
// (sphere.rs:57-98, plane.rs:59-84, triangle.rs:51-94, cube.rs:89-102).
__device__ __forceinline__ Hit hit_attrs_w(const DevScene& S, const ShapeW& R, uint32_t key, V3 o, V3 d,
                                           bool need_sphere_tex) {
    Hit h;
    h.mat = R.mat();
    const float4 r0 = R.w[1], r1 = R.w[2], r2 = R.w[3];
    h.eye = neg(norm(d));
    h.tu = 0.f;
    h.tv = 0.f;
    const int32_t kind = R.kind();
    if (kind == RT_SHAPE_SPHERE) {
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
            // glibc's atan2f / acosf (rt_libmf.hpp), as Rust's f32::atan2 / f32::acos call
            h.tu = (1.f + rtlibm::atan2f_fd(n.z, n.x) / PI_F) * 0.5f;
            h.tv = rtlibm::acosf_fd(n.y) / PI_F;
        }
    } else if (kind == RT_SHAPE_PLANE) {
        V3 to = pt_mul(r0, r1, r2, o);
        V3 td = vec3_mul(r0, r1, r2, d);
        V3 pn = v3(R.a(0), R.a(1), R.a(2));
        V3 po = v3(R.a(3), R.a(4), R.a(5));
        float t = 0.f;
        plane_t(to, td, pn, po, t);
        h.t = t;
        h.entering = t >= 0.f;
        h.p = add(o, mul(d, t));
        h.n = v3(R.a(6), R.a(7), R.a(8));  // transform * normal, evaluated on the host
        h.tu = dot(v3(R.a(9), R.a(10), R.a(11)), h.p);
        h.tv = dot(v3(R.a(12), R.a(13), R.a(14)), h.p);
    } else if (kind == RT_SHAPE_TRIANGLE) {
        float t = 0.f, u = 0.f, v = 0.f, det = 0.f;
        tri_hit(o, d, v3(R.a(0), R.a(1), R.a(2)), v3(R.a(3), R.a(4), R.a(5)), v3(R.a(6), R.a(7), R.a(8)),
                t, u, v, det);
        h.t = t;
        h.p = add(o, mul(d, t));
        h.n = v3(R.a(9), R.a(10), R.a(11));
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
__device__ __forceinline__ Hit hit_attrs(const DevScene& S, uint32_t key, V3 o, V3 d, bool need_sphere_tex) {
    return hit_attrs_w(S, load_shape(S.shapes, key >> 4), key, o, d, need_sphere_tex);
}

// Saturating f32 -> i32 cast (Rust `as i32`: NaN -> 0)
__device__ __forceinline__ int32_t sat_i32(float x) {
    if (x != x) return 0;
    if (x >= 2147483648.f) return 2147483647;
    if (x <= -2147483648.f) return (int32_t)0x80000000u;
    return (int32_t)x;
}

// Color::as_u8 (color.rs:43-46): (255 * c) as u8 -- truncating, saturating, NaN -> 0
__device__ __forceinline__ uint8_t as_u8(float c) {
    const float x = 255.f * c;
    uint8_t q = 0;
    if (x > 0.f) q = (x >= 255.f) ? (uint8_t)255 : (uint8_t)x;
    return q;
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
// with h = norm(norm(eye) + norm(l)); ne = norm(eye), the same for every light of a node,
// is evaluated once by the caller (reflected_energy_ne).
__device__ __forceinline__ V3 reflected_energy_ne(V3 E, V3 l, V3 n, V3 ne, V3 kd, V3 ks, float power) {
    float ln = dot(l, n);
    V3 hv = norm(add(ne, norm(l)));
    float mh = dot(n, hv);
    V3 spec = v3(0.f, 0.f, 0.f);
    if (!(mh < 0.f)) {
        float pw = RT_POW(mh, power);  // material.rs:211, glibc's powf
        spec = v3((pw * E.x) * ks.x, (pw * E.y) * ks.y, (pw * E.z) * ks.z);
    }
    return v3((ln * E.x) * kd.x + spec.x, (ln * E.y) * kd.y + spec.y, (ln * E.z) * kd.z + spec.z);
}
__device__ __forceinline__ V3 reflected_energy(V3 E, V3 l, const Hit& h, V3 kd, V3 ks, float power) {
    return reflected_energy_ne(E, l, h.n, norm(h.eye), kd, ks, power);
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

// reflect_ray's direction (render.rs:105-110, Vector3::reflect vector3.rs:113-115)
__device__ __forceinline__ V3 reflect_dir(V3 rd, V3 n) { return neg(norm(sub(mul(n, 2.f * dot(rd, n)), rd))); }

// refract_ray's direction (render.rs:112-125; not re-normalised); false = total internal
// reflection (None)
__device__ __forceinline__ bool refract_dir(V3 rd, V3 n, float n1, float n2, V3& trd) {
    float ratio = n1 / n2;
    float m_dot_r = -dot(rd, n);
    float cos2 = 1.f - ratio * ratio * (1.f - m_dot_r * m_dot_r);
    if (!(cos2 > 0.f)) return false;
    float ct = sqrtf(cos2);
    trd = add(mul(rd, ratio), mul(n, ratio * m_dot_r - ct));
    return true;
}

// The child weights of a hit node (render.rs:70-98), from what the trace pass stores
// (ray direction, normal) and the material: the same expressions the trace pass uses for
// the child rays, so the combine pass re-evaluates them bit for bit.  f.flags gets F_REFL
// / F_SPEC / F_REFR / F_TIR; the caller fills the ambient + lights and kd / ks.
__device__ __forceinline__ void node_weights(const MatRec& M, V3 rd, V3 n, V3 ne, float n1, float n2, Frame& f) {
    f.flags = 0u;
    f.fr = f.dr = f.pw = f.ft = 0.f;
    if (M.reflectivity > RT_EPS) {
        f.flags |= F_REFL;
        const V3 rrd = reflect_dir(rd, n);
        f.fr = fresnel_reflection(rrd, n, n1, n2);
        f.dr = dot(rrd, n);
        const V3 hv = norm(add(ne, norm(rrd)));  // ne = norm(eye_dir)
        const float mh = dot(n, hv);
        if (!(mh < 0.f)) {
            f.flags |= F_SPEC;
            f.pw = RT_POW(mh, M.power);
        }
    }
    if (M.refraction_index > RT_EPS) {
        f.flags |= F_REFR;
        V3 trd;
        if (refract_dir(rd, n, n1, n2, trd))
            f.ft = 1.f - fresnel_reflection(trd, neg(n), n1, n2);
        else
            f.flags |= F_TIR;
    }
}

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

}  // namespace rtdev
