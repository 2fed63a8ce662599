// rt_scan.hpp -- the nearest-hit scan of Scene::intersect (scene/mod.rs:98-116), the
// hot loop of the megakernel.  Included by rt_kernels.hip.
//
// Every lane scans the whole primitive list for its own ray; the list is walked with
// wave-uniform indices, so primitive records arrive through SMEM into SGPRs and are
// prefetched one group ahead (the s_load of group i+1 is in flight while group i
// computes).  Two throughput devices, both bit-exact w.r.t. the reference arithmetic:
//
//  * 2-wide packed f32 (v_pk_mul_f32 / v_pk_add_f32): spheres and loose triangles are
//    stored and tested in pairs, each packed instruction evaluating the same reference
//    expression for two primitives.  Packed f32 ops round exactly like their scalar
//    forms, so each lane of the pair computes what the reference computes.
//  * Compile-time cube triangles: the 12 object-space triangles of Cube::new
//    (cube.rs:21-77) have edges with components in {-1, 0, 1}.  Möller–Trumbore is
//    instantiated per triangle with those constants as types (`Zero`, `One`, `MinusOne`):
//    x*1 -> x, x*(-1) -> -x (exact), and terms x*0 are dropped, which changes at most the
//    SIGN of a zero result -- never a non-zero value and never the outcome of any of the
//    reference's comparisons (< 0, > 1, |det| < EPS all treat +0 and -0 alike).
#pragma once
// (included inside namespace rtdev, after the V3 helpers of rt_kernels.hip)

// RT_DIAG builds (tools only) count, per wave, how often each divergent hit path of the
// scan is entered; the counts go to rt_scan_stats (see tools/scan_stats.py).
#ifndef RT_DIAG
#define RT_DIAG 0
#endif
#if RT_DIAG
__device__ unsigned long long rt_scan_stats[40];
#define RT_STAT(i) do { if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == \
    (uint32_t)__builtin_ctzll(__ballot(1))) atomicAdd(&rt_scan_stats[i], 1ull); } while (0)
#else
#define RT_STAT(i) do { } while (0)
#endif
#ifndef RT_TASK_CLOCK
#define RT_TASK_CLOCK 0
#endif
#if RT_TASK_CLOCK
#define RT_SHADOW_CLOCK_WORDS (2u + 4u * (1u << 20))
__device__ uint32_t rt_shadow_clock[RT_SHADOW_CLOCK_WORDS];
// trace kernels: per level (< 16) a header of 4 words (tasks' entries, grid waves, task width)
// and 2^16 task records of 4 words
#define RT_TRACE_CLOCK_TASKS (1u << 16)
#define RT_TRACE_CLOCK_WORDS (16u * (4u + 4u * RT_TRACE_CLOCK_TASKS))
__device__ uint32_t rt_trace_clock[RT_TRACE_CLOCK_WORDS];
#endif

typedef float f2 __attribute__((ext_vector_type(2)));
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(3))) float4 lfloat4;
#else
typedef const float4 lfloat4;
#endif

__device__ __forceinline__ f2 bc(float x) { return f2{x, x}; }

// ------------------------------------------------------------------ zero-typed algebra
struct Zero {};
struct One {};
struct MinusOne {};
template <int C> struct Unit { typedef Zero type; };
template <> struct Unit<1> { typedef One type; };
template <> struct Unit<-1> { typedef MinusOne type; };

__device__ __forceinline__ float mul_(float a, float b) { return a * b; }
__device__ __forceinline__ Zero mul_(float, Zero) { return Zero{}; }
__device__ __forceinline__ Zero mul_(Zero, float) { return Zero{}; }
__device__ __forceinline__ Zero mul_(Zero, Zero) { return Zero{}; }
__device__ __forceinline__ float mul_(float a, One) { return a; }
__device__ __forceinline__ float mul_(One, float a) { return a; }
__device__ __forceinline__ float mul_(float a, MinusOne) { return -a; }
__device__ __forceinline__ float mul_(MinusOne, float a) { return -a; }
__device__ __forceinline__ Zero mul_(Zero, One) { return Zero{}; }
__device__ __forceinline__ Zero mul_(Zero, MinusOne) { return Zero{}; }
__device__ __forceinline__ Zero mul_(One, Zero) { return Zero{}; }
__device__ __forceinline__ Zero mul_(MinusOne, Zero) { return Zero{}; }

__device__ __forceinline__ float add_(float a, float b) { return a + b; }
__device__ __forceinline__ float add_(float a, Zero) { return a; }
__device__ __forceinline__ float add_(Zero, float b) { return b; }
__device__ __forceinline__ Zero add_(Zero, Zero) { return Zero{}; }
__device__ __forceinline__ float sub_(float a, float b) { return a - b; }
__device__ __forceinline__ float sub_(float a, Zero) { return a; }
__device__ __forceinline__ float sub_(Zero, float b) { return -b; }
__device__ __forceinline__ Zero sub_(Zero, Zero) { return Zero{}; }
__device__ __forceinline__ float val_(float a) { return a; }
__device__ __forceinline__ float val_(Zero) { return 0.f; }

// Möller–Trumbore (triangle.rs:51-80) on one cube triangle: v0 = 0.5 * (SX, SY, SZ),
// e1 = (A, B, C), e2 = (D, E, F), all compile-time.  Same expression tree as tri_hit.
template <int SX, int SY, int SZ, int A, int B, int C, int D, int E, int F>
__device__ __forceinline__ void cube_tri(V3 o, V3 d, uint32_t key, float& bt, uint32_t& bk) {
    typename Unit<A>::type e1x; typename Unit<B>::type e1y; typename Unit<C>::type e1z;
    typename Unit<D>::type e2x; typename Unit<E>::type e2y; typename Unit<F>::type e2z;
    // pvec = d x e2
    auto px = sub_(mul_(d.y, e2z), mul_(d.z, e2y));
    auto py = sub_(mul_(d.z, e2x), mul_(d.x, e2z));
    auto pz = sub_(mul_(d.x, e2y), mul_(d.y, e2x));
    float det = val_(add_(add_(mul_(e1x, px), mul_(e1y, py)), mul_(e1z, pz)));
    if (fabsf(det) < RT_EPS) return;
    // tvec = o - v0
    float tx = o.x - 0.5f * (float)SX, ty = o.y - 0.5f * (float)SY, tz = o.z - 0.5f * (float)SZ;
    float un = val_(add_(add_(mul_(tx, px), mul_(ty, py)), mul_(tz, pz)));
    float adet = fabsf(det);
    bool opp = (un < 0.f) != (det < 0.f);
    bool early = (adet <= 1048576.f) &&
                 ((opp && (un != 0.f) && (fabsf(un) >= 1.17549435e-38f)) || (fabsf(un) > 2.f * adet));
    if (early) return;
    RT_STAT(4);
    float inv_det = 1.0f / det;
    float u = un * inv_det;
    if (u < 0.f || u > 1.f) return;
    // qvec = tvec x e1
    auto qx = sub_(mul_(ty, e1z), mul_(tz, e1y));
    auto qy = sub_(mul_(tz, e1x), mul_(tx, e1z));
    auto qz = sub_(mul_(tx, e1y), mul_(ty, e1x));
    float v = val_(add_(add_(mul_(d.x, qx), mul_(d.y, qy)), mul_(d.z, qz))) * inv_det;
    if (v < 0.f || u + v > 1.f) return;
    float t = val_(add_(add_(mul_(e2x, qx), mul_(e2y, qy)), mul_(e2z, qz))) * inv_det;
    if (t < 0.f) return;
    take(t, key, bt, bk);
}

// The 12 triangles in the inner scene's order (cube.rs:58-69); v0 signs and edges
// follow Triangle::new(verts) with e1 = v[1]-v[0], e2 = v[2]-v[0].  rt_scene_create
// checks this table against the host-computed one (rt_cube_table_check).
#define RT_CUBE_TRIS(X)                                  \
    X(0, 1, -1, -1, -1, 0, 0, -1, 1, 0)   /* tf1 v1 v2 v3 */ \
    X(1, 1, 1, -1, 0, -1, 0, -1, 0, 0)    /* tf2 v0 v1 v3 */ \
    X(2, 1, -1, 1, -1, 1, 0, 0, 1, 0)     /* tk1 v7 v5 v4 */ \
    X(3, -1, 1, 1, 1, -1, 0, 0, -1, 0)    /* tk2 v5 v7 v6 */ \
    X(4, 1, 1, -1, 0, 0, 1, 0, -1, 1)     /* tr1 v0 v4 v7 */ \
    X(5, 1, -1, 1, 0, 0, -1, 0, 1, -1)    /* tr2 v7 v1 v0 */ \
    X(6, -1, 1, 1, 0, 0, -1, 0, -1, 0)    /* tl1 v5 v3 v6 */ \
    X(7, -1, -1, 1, 0, 1, -1, 0, 0, -1)   /* tl2 v6 v3 v2 */ \
    X(8, -1, 1, 1, 1, 0, 0, 1, 0, -1)     /* tt1 v5 v4 v0 */ \
    X(9, 1, 1, -1, -1, 0, 0, -1, 0, 1)    /* tt2 v0 v3 v5 */ \
    X(10, 1, -1, -1, 0, 0, 1, -1, 0, 1)   /* tb1 v1 v7 v6 */ \
    X(11, -1, -1, 1, 0, 0, -1, 1, 0, -1)  /* tb2 v6 v2 v1 */

__device__ __forceinline__ void cube_scan(V3 to, V3 td, uint32_t key0, float& bt, uint32_t& bk) {
#define RT_CUBE_CALL(k, sx, sy, sz, a, b, c, d_, e, f) \
    cube_tri<sx, sy, sz, a, b, c, d_, e, f>(to, td, key0 | (uint32_t)(k), bt, bk);
    RT_CUBE_TRIS(RT_CUBE_CALL)
#undef RT_CUBE_CALL
}

// ------------------------------------------------------------------ sphere tail
// sphere.rs:126-145 after the discriminant: returns t for a non-negative discriminant
__device__ __forceinline__ bool sphere_finish(float a, float b, float c, float discr, float& t_out) {
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
    return true;
}

// triangle.rs:61-80 for a lane whose det passed and whose u-numerator survived the
// pre-test
__device__ __forceinline__ bool tri_finish(V3 d, V3 tv, V3 e1, V3 e2, float det, float un, float& t_out) {
    float inv_det = 1.0f / det;
    float u = un * inv_det;
    if (u < 0.f || u > 1.f) return false;
    V3 q = cross(tv, e1);
    float v = dot(d, q) * inv_det;
    if (v < 0.f || u + v > 1.f) return false;
    float t = dot(e2, q) * inv_det;
    if (t < 0.f) return false;
    t_out = t;
    return true;
}

__device__ __forceinline__ bool tri_early(float det, float un) {
    float adet = fabsf(det);
    bool opp = (un < 0.f) != (det < 0.f);
    return (adet <= 1048576.f) &&
           ((opp && (un != 0.f) && (fabsf(un) >= 1.17549435e-38f)) || (fabsf(un) > 2.f * adet));
}

// ------------------------------------------------------------------ record views
// Pair records (64 B / 96 B) are read as float4 groups from the constant address space.
struct SphPair {  // 16 floats
    float4 q0, q1, q2, q3;
};
struct TriPair {  // 24 floats
    float4 q0, q1, q2, q3, q4, q5;
};
struct Rec16 {  // a general sphere or cube: inverse rows 0..2 + key
    float4 r0, r1, r2, rk;
};

__device__ __forceinline__ SphPair ld_sph(cfloat4* p) { return SphPair{p[0], p[1], p[2], p[3]}; }
__device__ __forceinline__ TriPair ld_tri(cfloat4* p) { return TriPair{p[0], p[1], p[2], p[3], p[4], p[5]}; }
__device__ __forceinline__ Rec16 ld_rec(cfloat4* p) { return Rec16{p[0], p[1], p[2], p[3]}; }

// diag sphere pair: {sxA sxB syA syB} {szA szB oxA oxB} {oyA oyB ozA ozB} {keyA keyB - -}
__device__ __forceinline__ void sph_pair(const SphPair& R, V3 o, V3 d, float& bt, uint32_t& bk) {
    f2 sx = f2{R.q0.x, R.q0.y}, sy = f2{R.q0.z, R.q0.w}, sz = f2{R.q1.x, R.q1.y};
    f2 ox = f2{R.q1.z, R.q1.w}, oy = f2{R.q2.x, R.q2.y}, oz = f2{R.q2.z, R.q2.w};
    // translate*scale inverse: pt_mul / vec3_mul with the zero off-diagonal terms dropped
    f2 tox = bc(o.x) * sx + ox, toy = bc(o.y) * sy + oy, toz = bc(o.z) * sz + oz;
    f2 tdx = bc(d.x) * sx, tdy = bc(d.y) * sy, tdz = bc(d.z) * sz;
    f2 a = (tdx * tdx + tdy * tdy) + tdz * tdz;
    f2 b = 2.f * ((tdx * tox + tdy * toy) + tdz * toz);
    f2 c = ((tox * tox + toy * toy) + toz * toz) - 1.f;
    f2 discr = b * b - (4.f * a) * c;
    bool hA = !(discr.x < 0.f), hB = !(discr.y < 0.f);
    if (hA || hB) {
        RT_STAT(1);
        float t;
        if (hA && sphere_finish(a.x, b.x, c.x, discr.x, t)) take(t, keyof(R.q3.x), bt, bk);
        if (hB && sphere_finish(a.y, b.y, c.y, discr.y, t)) take(t, keyof(R.q3.y), bt, bk);
    }
}

// general sphere: full pt_mul / vec3_mul with the inverse rows
__device__ __forceinline__ void sph_general(const Rec16& R, V3 o, V3 d, float& bt, uint32_t& bk) {
    V3 to = pt_mul(R.r0, R.r1, R.r2, o);
    V3 td = vec3_mul(R.r0, R.r1, R.r2, d);
    float a = len2(td);
    float b = 2.f * dot(td, to);
    float c = len2(to) - 1.f;
    float discr = b * b - 4.f * a * c;
    float t;
    if (!(discr < 0.f)) {
        RT_STAT(2);
        if (sphere_finish(a, b, c, discr, t)) take(t, keyof(R.rk.x), bt, bk);
    }
}

// loose triangle pair: {v0xA v0xB v0yA v0yB} {v0zA v0zB e1xA e1xB} {e1yA e1yB e1zA e1zB}
//                      {e2xA e2xB e2yA e2yB} {e2zA e2zB keyA keyB} {- - - -}
__device__ __forceinline__ void tri_pair(const TriPair& R, V3 o, V3 d, float& bt, uint32_t& bk) {
    f2 v0x = f2{R.q0.x, R.q0.y}, v0y = f2{R.q0.z, R.q0.w}, v0z = f2{R.q1.x, R.q1.y};
    f2 e1x = f2{R.q1.z, R.q1.w}, e1y = f2{R.q2.x, R.q2.y}, e1z = f2{R.q2.z, R.q2.w};
    f2 e2x = f2{R.q3.x, R.q3.y}, e2y = f2{R.q3.z, R.q3.w}, e2z = f2{R.q4.x, R.q4.y};
    // pvec = d x e2; det = e1 . pvec; tvec = o - v0; un = tvec . pvec
    f2 px = bc(d.y) * e2z - bc(d.z) * e2y;
    f2 py = bc(d.z) * e2x - bc(d.x) * e2z;
    f2 pz = bc(d.x) * e2y - bc(d.y) * e2x;
    f2 det = (e1x * px + e1y * py) + e1z * pz;
    f2 tx = bc(o.x) - v0x, ty = bc(o.y) - v0y, tz = bc(o.z) - v0z;
    f2 un = (tx * px + ty * py) + tz * pz;
    bool aA = !(fabsf(det.x) < RT_EPS) && !tri_early(det.x, un.x);
    bool aB = !(fabsf(det.y) < RT_EPS) && !tri_early(det.y, un.y);
    if (aA || aB) {
        RT_STAT(3);
        float t;
        if (aA && tri_finish(d, v3(tx.x, ty.x, tz.x), v3(e1x.x, e1y.x, e1z.x), v3(e2x.x, e2y.x, e2z.x), det.x,
                             un.x, t))
            take(t, keyof(R.q4.z), bt, bk);
        if (aB && tri_finish(d, v3(tx.y, ty.y, tz.y), v3(e1x.y, e1y.y, e1z.y), v3(e2x.y, e2y.y, e2z.y), det.y,
                             un.y, t))
            take(t, keyof(R.q4.w), bt, bk);
    }
}

// plane (plane.rs:59-66) with its own inverse: {inv r0} {inv r1} {inv r2} {n key} {origin -}
__device__ __forceinline__ void plane_one(cfloat4* r, V3 o, V3 d, float& bt, uint32_t& bk) {
    float4 r0 = r[0], r1 = r[1], r2 = r[2], rn = r[3], ro = r[4];
    V3 to = pt_mul(r0, r1, r2, o);
    V3 td = vec3_mul(r0, r1, r2, d);
    float t;
    if (plane_t(to, td, xyz(rn), xyz(ro), t)) take(t, keyof(rn.w), bt, bk);
}

// ------------------------------------------------------------------ test counters
// Lane-weighted counts of every test the scan runs (RT_OPS_*): wave-uniform, kept in
// SGPRs, added to DevScene::scan_ops once per wave when a kernel ends.
struct ScanCnt {
    static constexpr bool kCount = true;
    uint32_t node, dsph, gsph, tri, cube_box, cube, graze, plane, graze_n;
    uint32_t cyc_node, cyc_leaf, cyc_graze, cyc_scan, cyc_load, cyc_post, cyc_self;
};
__device__ __forceinline__ uint32_t rt_clock() { return (uint32_t)__builtin_amdgcn_s_memtime(); }
// The uncounted variant: the same expressions, every `+=` a no-op (compiled away).
struct NoCntField {
    __device__ NoCntField& operator+=(uint32_t) { return *this; }
};
struct NoCnt {
    static constexpr bool kCount = false;
    NoCntField node, dsph, gsph, tri, cube_box, cube, graze, plane, graze_n;
    NoCntField cyc_node, cyc_leaf, cyc_graze, cyc_scan, cyc_load, cyc_post, cyc_self;
};
// cycle accounting of the instrumented variant (compiled away otherwise)
#define RT_T0(C, v) uint32_t v = 0; if constexpr (C::kCount) v = rt_clock()
#define RT_T1(C, c, f, v) do { if constexpr (C::kCount) (c).f += rt_clock() - (v); } while (0)
__device__ __forceinline__ void cnt_init(ScanCnt& c) {
    c.node = c.dsph = c.gsph = c.tri = c.cube_box = c.cube = c.graze = c.plane = c.graze_n = 0;
    c.cyc_node = c.cyc_leaf = c.cyc_graze = c.cyc_scan = c.cyc_load = c.cyc_post = c.cyc_self = 0;
}
__device__ __forceinline__ uint32_t active_lanes() { return (uint32_t)__builtin_popcountll(__ballot(1)); }
#define RT_OPS(c, f) ((c).f += active_lanes())
__device__ __forceinline__ void cnt_add(unsigned long long* p, uint32_t v) {
    if (v) atomicAdd(p, (unsigned long long)v);
}
// Adds the wave's counts to `dst` (RT_OPS_N counters) from one lane.
__device__ __forceinline__ void cnt_flush(const ScanCnt& c, unsigned long long* dst) {
    uint64_t m = __ballot(1);
    if (m == 0) return;
    if (__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) == 0) {
        cnt_add(dst + RT_OPS_NODE, c.node);
        cnt_add(dst + RT_OPS_DSPH, c.dsph);
        cnt_add(dst + RT_OPS_GSPH, c.gsph);
        cnt_add(dst + RT_OPS_TRI, c.tri);
        cnt_add(dst + RT_OPS_CUBE_BOX, c.cube_box);
        cnt_add(dst + RT_OPS_CUBE, c.cube);
        cnt_add(dst + RT_OPS_GRAZE, c.graze);
        cnt_add(dst + RT_OPS_PLANE, c.plane);
        cnt_add(dst + RT_OPS_GRAZE_N, c.graze_n);
    }
}
__device__ __forceinline__ unsigned long long* ops_slot(const DevScene& S) {
    return S.scan_ops + (blockIdx.x % RT_OPS_SLOTS) * RT_OPS_STRIDE;
}

// Leaf loops load record i + 1 while testing record i (loading each record at the top of its
// iteration instead: 4.65 vs 4.62 ms, round 1)
#define RT_PF_INIT(T, ld, p) T cur = ld(p);
#define RT_PF_NEXT(T, ld, p, K) \
    p += K;                     \
    T nxt = ld(p);
#define RT_PF_ADV cur = nxt;

// ------------------------------------------------------------------ linear runs
// Group loops prefetch record i+1 before testing record i; every section is padded by
// one group so the look-ahead load stays inside the allocation.
// The hierarchy's sphere pairs staged in LDS by the walk kernels (ldsph: their copy of
// records [0, n_dsph_bvh), which every hierarchy leaf's run lies in): every lane reads the
// same address (a broadcast) and the packed tests take the record from VGPRs.  No misses,
// unlike the scalar data cache, which the light-buffer copies and the rest of the scene
// share (+1.4%; reading the next record ahead, or moving it to SGPRs by readfirstlane, lost).
__device__ __forceinline__ SphPair ld_sph_l(lfloat4* p) { return SphPair{p[0], p[1], p[2], p[3]}; }
template <class C>
__device__ __forceinline__ void run_dsph_lds(int b, int e, V3 o, V3 d, float& bt, uint32_t& bk, C& c,
                                             lfloat4* ldsph) {
    lfloat4* p = ldsph + 4 * b;
    for (int i = b; i < e; ++i, p += 4) {
        RT_OPS(c, dsph);
        sph_pair(ld_sph_l(p), o, d, bt, bk);
    }
}
template <class C>
__device__ __forceinline__ void run_dsph(const DevScene& S, int b, int e, V3 o, V3 d, float& bt, uint32_t& bk,
                                         C& c) {
    if (b >= e) return;
    cfloat4* p = cptr(S.dsph) + 4 * b;
    RT_PF_INIT(SphPair, ld_sph, p)
    for (int i = b; i < e; ++i) {
        RT_PF_NEXT(SphPair, ld_sph, p, 4)
        RT_OPS(c, dsph);
        sph_pair(cur, o, d, bt, bk);
        RT_PF_ADV
    }
}
template <class C>
__device__ __forceinline__ void run_gsph(const DevScene& S, int b, int e, V3 o, V3 d, float& bt, uint32_t& bk,
                                         C& c) {
    if (b >= e) return;
    cfloat4* p = cptr(S.gsph) + 4 * b;
    RT_PF_INIT(Rec16, ld_rec, p)
    for (int i = b; i < e; ++i) {
        RT_PF_NEXT(Rec16, ld_rec, p, 4)
        RT_OPS(c, gsph);
        sph_general(cur, o, d, bt, bk);
        RT_PF_ADV
    }
}
template <class C>
__device__ __forceinline__ void run_tri(const DevScene& S, int b, int e, V3 o, V3 d, float& bt, uint32_t& bk,
                                        C& c) {
    if (b >= e) return;
    cfloat4* p = cptr(S.tri) + 6 * b;
    RT_PF_INIT(TriPair, ld_tri, p)
    for (int i = b; i < e; ++i) {
        RT_PF_NEXT(TriPair, ld_tri, p, 6)
        RT_OPS(c, tri);
        tri_pair(cur, o, d, bt, bk);
        RT_PF_ADV
    }
}
template <class C>
__device__ __forceinline__ void run_cube(const DevScene& S, int b, int e, V3 o, V3 d, float& bt, uint32_t& bk,
                                         C& c) {
    if (b >= e) return;
    cfloat4* p = cptr(S.cube) + 4 * b;
    RT_PF_INIT(Rec16, ld_rec, p)
    for (int i = b; i < e; ++i) {
        RT_PF_NEXT(Rec16, ld_rec, p, 4)
        RT_OPS(c, cube);
        V3 to = pt_mul(cur.r0, cur.r1, cur.r2, o);
        V3 td = vec3_mul(cur.r0, cur.r1, cur.r2, d);
        cube_scan(to, td, keyof(cur.rk.x), bt, bk);
        RT_PF_ADV
    }
}

// ------------------------------------------------------------------ culling hierarchy
// DESIGN.md "Exact culling".  For a ray (o, d) and D = |o - c| + r (the ball (c, r)
// holds every hierarchy primitive), every hit the reference's f32 tests can report at t'
// satisfies: the point o + t*d lies within h(D) = (g2 D + g1) D + g0 of the primitive for
// some t* with |t' - t*| <= m(D)/|d|.  Every primitive's bound is on the reported point
// itself (t* = t', m = 0 today); triangles for rays meeting their plane at
// sin(phi) >= sin(phi_T), the triangle's own grazing threshold (rt_build.cpp graze_sin).
// h also covers the rounding of this slab test.  A child box is skipped for a lane only
// when its box grown by h misses the ray on [-m, t_max + m] (t_max = the lane's best t,
// or the shadow limit); the wave skips it only when every lane does.  Spheres,
// triangles and cubes never report t < 0; a lane already holding a plane hit at t < 0
// votes for nothing (nothing can beat a negative t).  Grazing rays: the grazing pass
// below tests exactly every hierarchy triangle whose plane some lane grazes.
__shared__ uint32_t rt_bvh_stack[4 * 32];  // one 32-entry stack per wave (256-thread blocks)

__device__ __forceinline__ float safe_rcp(float x) {
    float s = (fabsf(x) < 1e-30f) ? copysignf(1e-30f, x) : x;
    return __builtin_amdgcn_rcpf(s);
}
__device__ __forceinline__ float rfl(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

struct BvhRay {
    float ix, iy, iz;      // 1/d
    float pax, pay, paz;   // (o + h) / d
    float pbx, pby, pbz;   // (o - h) / d
    float on;              // |o|
    float m;               // t-margin m(D) / |d|
};

__device__ __forceinline__ BvhRay bvh_ray(const DevScene& S, V3 o, V3 d) {
    BvhRay R;
    float dx = o.x - S.bvh_cx, dy = o.y - S.bvh_cy, dz = o.z - S.bvh_cz;
    float D = sqrtf(dx * dx + dy * dy + dz * dz) + S.bvh_r;
    float h = fmaf(fmaf(S.bvh_g2, D, S.bvh_g1), D, S.bvh_g0);
    R.ix = safe_rcp(d.x);
    R.iy = safe_rcp(d.y);
    R.iz = safe_rcp(d.z);
    R.pax = (o.x + h) * R.ix;
    R.pay = (o.y + h) * R.iy;
    R.paz = (o.z + h) * R.iz;
    R.pbx = (o.x - h) * R.ix;
    R.pby = (o.y - h) * R.iy;
    R.pbz = (o.z - h) * R.iz;
    R.on = sqrtf(o.x * o.x + o.y * o.y + o.z * o.z);
    R.m = fmaf(S.bvh_m1, D, S.bvh_m0) / sqrtf(d.x * d.x + d.y * d.y + d.z * d.z) * 1.0001f;
    return R;
}

// both children of a node, 2-wide: {loA.x loB.x loA.y loB.y} {loA.z loB.z hiA.x hiB.x}
// {hiA.y hiB.y hiA.z hiB.z}
__device__ __forceinline__ void node_test(float4 q0, float4 q1, float4 q2, BvhRay R, float tmax, bool& hA,
                                          bool& hB) {
    f2 lx = f2{q0.x, q0.y}, ly = f2{q0.z, q0.w}, lz = f2{q1.x, q1.y};
    f2 ux = f2{q1.z, q1.w}, uy = f2{q2.x, q2.y}, uz = f2{q2.z, q2.w};
    f2 ax = __builtin_elementwise_fma(lx, bc(R.ix), -bc(R.pax));
    f2 ay = __builtin_elementwise_fma(ly, bc(R.iy), -bc(R.pay));
    f2 az = __builtin_elementwise_fma(lz, bc(R.iz), -bc(R.paz));
    f2 bx = __builtin_elementwise_fma(ux, bc(R.ix), -bc(R.pbx));
    f2 by = __builtin_elementwise_fma(uy, bc(R.iy), -bc(R.pby));
    f2 bz = __builtin_elementwise_fma(uz, bc(R.iz), -bc(R.pbz));
    const float tmin = -R.m;
    float enA = fmaxf(fmaxf(fminf(ax.x, bx.x), fminf(ay.x, by.x)), fmaxf(fminf(az.x, bz.x), tmin));
    float exA = fminf(fminf(fmaxf(ax.x, bx.x), fmaxf(ay.x, by.x)), fminf(fmaxf(az.x, bz.x), tmax));
    float enB = fmaxf(fmaxf(fminf(ax.y, bx.y), fminf(ay.y, by.y)), fmaxf(fminf(az.y, bz.y), tmin));
    float exB = fminf(fminf(fmaxf(ax.y, bx.y), fmaxf(ay.y, by.y)), fminf(fmaxf(az.y, bz.y), tmax));
    hA = enA <= exA;
    hB = enB <= exB;
}

// A cube of a leaf: its object-space box [-1/2 - hc, 1/2 + hc]^3 first (hc bounds how
// far a reported object-space hit point can lie outside the unit cube, measured by
// tools/cull_bounds_check.py, x32), then the 12 triangles if any lane can hit.
template <class C>
__device__ __forceinline__ void cube_culled(const Rec16& Rc, V3 o, V3 d, float on, float tmax, float& bt,
                                            uint32_t& bk, C& c) {
    V3 to = pt_mul(Rc.r0, Rc.r1, Rc.r2, o);
    V3 td = vec3_mul(Rc.r0, Rc.r1, Rc.r2, d);
    float m = fmaxf(fabsf(to.x), fmaxf(fabsf(to.y), fabsf(to.z)));
    float hc = 32.f * RT_EPS * (2.f * m + 1.f + fmaf(Rc.rk.y, on, Rc.rk.z));
    float b = 0.5f + hc;
    float ix = safe_rcp(td.x), iy = safe_rcp(td.y), iz = safe_rcp(td.z);
    float ax = (-b - to.x) * ix, bx = (b - to.x) * ix;
    float ay = (-b - to.y) * iy, by = (b - to.y) * iy;
    float az = (-b - to.z) * iz, bz = (b - to.z) * iz;
    float en = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.f));
    float ex = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tmax));
    RT_OPS(c, cube_box);
    if (__ballot(en <= ex)) {
        RT_OPS(c, cube);
        cube_scan(to, td, keyof(Rc.rk.x), bt, bk);
    }
}

#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) uint4 cuint4;
#else
typedef const uint4 cuint4;
#endif

// One leaf: its runs of pairs / general spheres / triangle pairs / cubes.
template <class C>
__device__ __forceinline__ void bvh_leaf(const DevScene& S, uint32_t li, V3 o, V3 d, float on, float tmax,
                                         float& bt, uint32_t& bk, C& c, lfloat4* ldsph = nullptr) {
    // (the descriptor from LDS instead -- staged after the sphere pairs, a broadcast read and
    // 8 readfirstlanes -- measured flat: 1091.7 vs 1093.1 Mpixels/s in 4 pairs, profiles/r4l)
    cuint4* lp = (cuint4*)S.bvh_leaves + 2 * li;
    uint4 a = lp[0], b = lp[1];
    if (ldsph)  // a hierarchy leaf, in a kernel that staged the sphere pairs
        run_dsph_lds((int)a.x, (int)a.y, o, d, bt, bk, c, ldsph);
    else
        run_dsph(S, (int)a.x, (int)a.y, o, d, bt, bk, c);
    run_gsph(S, (int)a.z, (int)a.w, o, d, bt, bk, c);
    run_tri(S, (int)b.x, (int)b.y, o, d, bt, bk, c);
    if (b.z < b.w) {
        cfloat4* p = cptr(S.cube) + 4 * b.z;
        for (uint32_t i = b.z; i < b.w; ++i, p += 4) cube_culled(ld_rec(p), o, d, on, tmax, bt, bk, c);
    }
}

// "hit nearer than the light" for the current best t (the reference's test)
__device__ __forceinline__ bool shadow_hit(V3 o, V3 d, float bt, float l2) {
    if (!(bt < __builtin_huge_valf())) return false;
    return len2(sub(add(o, mul(d, bt)), o)) < l2;
}
// the lane's answer can no longer change
__device__ __forceinline__ bool shadow_decided(V3 o, V3 d, float bt, float l2) {
    return bt < 0.f || shadow_hit(o, d, bt, l2);
}

// Walk the hierarchy.  SHADOW: t_max also stops at the light (tlim) and decided lanes
// stop voting; the walk ends when every lane is decided.

// The LDS of the walk kernels' LDS variant: node records, then the grazing pairs' normals
// (per-lane grazing sets), then the hierarchy's sphere pairs
__device__ __forceinline__ lfloat4* lds_dsph(const DevScene& S, lfloat4* lnodes) {
    return lnodes + 4 * S.n_bvh_nodes + ((S.graze_lane && S.graze_res) ? 8 * S.n_graze_blk : 0);
}

// LDS: node records staged in LDS by the kernel (lnodes != null), else read via SMEM
// novote (shadow): the lane's hierarchy primitives are settled already (light buffer).
template <bool SHADOW, bool LDS, class C>
__device__ __forceinline__ void bvh_walk(const DevScene& S, V3 o, V3 d, float& bt, uint32_t& bk, float tlim,
                                         float l2, C& c, lfloat4* lnodes, bool novote = false) {
    const BvhRay R = bvh_ray(S, o, d);
#if RT_DIAG
    if (!SHADOW) {  // slots 23-28: trace walks' lanes by D / R in (0,3] (3,6] (6,12] (12,25] (25,50] (50,inf);
                    // 29-31: leaf visits of waves whose farthest lane is within 3 R / 12 R / beyond
        const float dx = o.x - S.bvh_cx, dy = o.y - S.bvh_cy, dz = o.z - S.bvh_cz;
        const float q = (sqrtf(dx * dx + dy * dy + dz * dz) + S.bvh_r) / S.bvh_r;
        const int b = q <= 3.f ? 0 : q <= 6.f ? 1 : q <= 12.f ? 2 : q <= 25.f ? 3 : q <= 50.f ? 4 : 5;
        const bool first = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) ==
                           (uint32_t)__builtin_ctzll(__ballot(1));
        for (int k = 0; k < 6; k++) {
            const uint64_t m = __ballot(b == k);
            if (m && first) atomicAdd(&rt_scan_stats[23 + k], (unsigned long long)__builtin_popcountll(m));
        }
    }
    uint32_t rt_far_class = 0;
    if (!SHADOW) {
        const float dx = o.x - S.bvh_cx, dy = o.y - S.bvh_cy, dz = o.z - S.bvh_cz;
        const float q = (sqrtf(dx * dx + dy * dy + dz * dz) + S.bvh_r) / S.bvh_r;
        rt_far_class = __ballot(q > 12.f) ? 2u : (__ballot(q > 3.f) ? 1u : 0u);
    }
#endif
#if RT_DIAG
    // leaf-major planning (DESIGN.md "Leaf-major trace pass"): the leaves a trace ray's own
    // box tests admit with no nearest-hit bound during the walk (its bound at the start:
    // infinite, or the enclosing sphere's exit) -- slot 32, rays in slot 33 -- and, after the
    // walk, with its final nearest hit as the bound -- slot 34
    auto lane_leaves = [&](float tb) {
        uint32_t lst[48];
        int lsp = 0;
        uint32_t c = S.bvh_root, nl = 0;
        const float tn = tb < 0.f ? -__builtin_huge_valf() : tb + R.m;
        for (;;) {
            if (c & BVH_LEAF) {
                nl++;
            } else {
                cfloat4* q = cptr(S.bvh_nodes) + 4 * c;
                bool a, b;
                node_test(q[0], q[1], q[2], R, tn, a, b);
                const uint32_t ca = __float_as_uint(q[3].x), cb = __float_as_uint(q[3].y);
                if (a && b && lsp < 48) {
                    lst[lsp++] = cb;
                    c = ca;
                    continue;
                }
                if (a) { c = ca; continue; }
                if (b) { c = cb; continue; }
            }
            if (lsp == 0) break;
            c = lst[--lsp];
        }
        return nl;
    };
    if (!SHADOW && !novote) {
        atomicAdd(&rt_scan_stats[32], (unsigned long long)lane_leaves(bt));
        atomicAdd(&rt_scan_stats[33], 1ull);
    }
#endif
    uint32_t* stk = rt_bvh_stack + ((threadIdx.x >> 6) << 5);
    uint32_t sp = 0;
    uint32_t cur = S.bvh_root;
    bool done = SHADOW ? (novote || shadow_decided(o, d, bt, l2)) : false;
#if RT_DIAG
    // lanes whose own box test admitted the current node (stats build only)
    __shared__ uint64_t rt_need_stack[4 * 32];
    uint64_t* nstk = rt_need_stack + ((threadIdx.x >> 6) << 5);
    uint64_t need = __ballot(1);
#define RT_NEED(x) x
#else
#define RT_NEED(x)
#endif
    for (;;) {
        // the lane's limit: its best t (a plane's t < 0 beats everything: no votes), the
        // light for shadow rays, nothing once decided
        float tmax = SHADOW ? (done ? -1.f : fminf(bt, tlim)) : (novote ? -1.f : bt);
        float tnode = (tmax < 0.f) ? -__builtin_huge_valf() : tmax + R.m;
        RT_T0(C, t_it);
        if (cur & BVH_LEAF) {
#if RT_DIAG
            {
                uint64_t act = __ballot(SHADOW ? !done : true);
                if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == (uint32_t)__builtin_ctzll(__ballot(1))) {
                    const int sb = SHADOW ? 8 : 5;  // trace walks: slots 5-7, shadow walks: 8-10
                    atomicAdd(&rt_scan_stats[sb], (unsigned long long)__builtin_popcountll(act));
                    atomicAdd(&rt_scan_stats[sb + 1], (unsigned long long)__builtin_popcountll(act & need));
                    atomicAdd(&rt_scan_stats[sb + 2], 1ull);
                    if (!SHADOW) atomicAdd(&rt_scan_stats[29 + rt_far_class], 1ull);
                }
            }
#endif
            bvh_leaf(S, cur & ~BVH_LEAF, o, d, R.on, tmax, bt, bk, c, LDS ? lds_dsph(S, lnodes) : nullptr);
            RT_T1(C, c, cyc_leaf, t_it);
            if (SHADOW) {
                done = novote || shadow_decided(o, d, bt, l2);
                if (__ballot(!done) == 0) break;
            }
        } else {
            float4 q0, q1, q2, q3;
            if (LDS) {
                lfloat4* q = lnodes + 4 * cur;
                q0 = q[0];
                q1 = q[1];
                q2 = q[2];
                q3 = q[3];
            } else {
                cfloat4* q = cptr(S.bvh_nodes) + 4 * cur;
                q0 = q[0];
                q1 = q[1];
                q2 = q[2];
                q3 = q[3];
            }
            bool hA, hB;
            node_test(q0, q1, q2, R, tnode, hA, hB);
            RT_OPS(c, node);
            bool anyA = __ballot(hA) != 0, anyB = __ballot(hB) != 0;
            uint32_t cA = __float_as_uint(q3.x), cB = __float_as_uint(q3.y);
            RT_T1(C, c, cyc_node, t_it);
            if (anyA && anyB) {
                uint32_t axis = __float_as_uint(q3.z);
                float da = rfl(axis == 0 ? d.x : (axis == 1 ? d.y : d.z));
                bool b_first = da < 0.f;  // child A holds the lower centroids
                RT_NEED(nstk[sp] = __ballot(b_first ? hA : hB); need = __ballot(b_first ? hB : hA);)
                stk[sp++] = b_first ? cA : cB;
                cur = b_first ? cB : cA;
                continue;
            }
            if (anyA) {
                RT_NEED(need = __ballot(hA);)
                cur = cA;
                continue;
            }
            if (anyB) {
                RT_NEED(need = __ballot(hB);)
                cur = cB;
                continue;
            }
        }
        if (sp == 0) break;
        RT_NEED(need = nstk[sp - 1];)
        cur = rfl(stk[--sp]);
    }
#if RT_DIAG
    if (!SHADOW && !novote) atomicAdd(&rt_scan_stats[34], (unsigned long long)lane_leaves(bt));
#endif
}

// cube-map cell of a direction (face = largest |component|, ties x > y > z); the host
// builds light buffers and grazing masks over the same cells (rt_build.cpp lb_face_dir)
// A wave-uniform scene constant read where it is used: the compiler may not hoist what is
// derived from it out of the loops.  Hoisted, such values (0.5 res, res - 1, 16 / r ...) were
// computed once into VGPRs, spilled to scratch, and every reload inside the trace iteration
// waited (vmcnt counts stores on gfx9) for the iteration's outstanding stores.
__device__ __forceinline__ uint32_t opaque_u(uint32_t x) {
    __asm__ volatile("" : "+s"(x));
    return x;
}
__device__ __forceinline__ float opaque_f(float x) {
    __asm__ volatile("" : "+s"(x));
    return x;
}
// ... and a per-lane value (loop-invariant values derived from it are recomputed per use)
__device__ __forceinline__ V3 opaque_v3(V3 v) {
    __asm__ volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z));
    return v;
}
__device__ __forceinline__ uint32_t lb_cell(uint32_t res, V3 v) {
    res = opaque_u(res);
    const float ax = fabsf(v.x), ay = fabsf(v.y), az = fabsf(v.z);
    uint32_t f;
    float a, b, m;
    if (ax >= ay && ax >= az) {
        f = v.x < 0.f ? 1u : 0u;
        a = v.y;
        b = v.z;
        m = ax;
    } else if (ay >= az) {
        f = v.y < 0.f ? 3u : 2u;
        a = v.x;
        b = v.z;
        m = ay;
    } else {
        f = v.z < 0.f ? 5u : 4u;
        a = v.x;
        b = v.y;
        m = az;
    }
    const float inv = __builtin_amdgcn_rcpf(m), hr = 0.5f * (float)res;
    const int i = min(max((int)((a * inv + 1.f) * hr), 0), (int)res - 1);
    const int j = min(max((int)((b * inv + 1.f) * hr), 0), (int)res - 1);
    return (f * res + (uint32_t)j) * res + (uint32_t)i;
}

// The light-buffer tier a shadow ray's origin falls in -- the first tier t with D <=
// lb_dmax 2^t and a light within RT_LB_LMAX 2^t (the buffers built for that reach and that
// direction error, rt_build.cpp build_light_buffers) -- or -1: no buffer (the light has none,
// or the origin lies beyond its tiers) -- walk.  LightRec::lb_base: the light's first cell in
// bits 0-27, its tier count in bits 28-30 (~0: no buffer).
// ... for the origin's D = |o - c| + R given (the trace kernel's queue keys: D once per hit)
__device__ __forceinline__ int lb_tier_at(const DevScene& S, uint32_t lb_base, float D, float l2) {
    if (!S.lb_res || lb_base == 0xFFFFFFFFu) return -1;
    const int tiers = (int)((lb_base >> 28) & 7u);
    float thr = S.lb_dmax, lm2 = RT_LB_LMAX * RT_LB_LMAX;
    for (int t = 0; t < tiers; t++, thr *= 2.f, lm2 *= 4.f)
        if (D <= thr && l2 <= lm2) return t;
    return -1;
}
__device__ __forceinline__ int lb_tier(const DevScene& S, uint32_t lb_base, V3 o, float l2) {
    const float dx = o.x - S.bvh_cx, dy = o.y - S.bvh_cy, dz = o.z - S.bvh_cz;
    return lb_tier_at(S, lb_base, sqrtf(dx * dx + dy * dy + dz * dz) + S.bvh_r, l2);
}

// Grazing pass: every hierarchy triangle whose plane some lane's ray meets at
// sin(phi) < 1.01 sin(phi_min) is tested exactly for the wave (the hierarchy's bounds
// do not cover it).  Triangles come in blocks of 8 with similar normals; a block whose
// normal cone no lane's direction can graze is skipped after one dot product.
// With direction cells (S.graze_res): the wave ORs the pair masks of its lanes' cells
// (a superset of the pairs any lane grazes) and runs the per-triangle test on those.
// The lane's first two mask words, loaded when its scan starts (latency hidden by the walk).
struct GrazePre {
    uint32_t m0, m1;
};
__device__ __forceinline__ GrazePre graze_prefetch(const DevScene& S, V3 d) {
    GrazePre g{0u, 0u};
    if (false && S.graze_res && S.n_graze_blk) {
        const uint32_t* mp = S.graze_mask + (size_t)lb_cell(S.graze_res, d) * S.graze_words;
        g.m0 = mp[0];
        if (S.graze_words > 1) g.m1 = mp[1];
    }
    return g;
}

// Per-lane sets (S.graze_lane): each lane first runs the per-triangle test on the pairs
// its own cell lists (normals from LDS when the kernel staged them after the node
// records, else per-lane loads); the wave then tests, by tri_pair, the union of the pairs
// some lane really grazes -- the same pairs the union path below ends up testing, without
// a round trip per candidate of the wave's union.  novote: the lane's answer is settled
// (a decided shadow ray), it lists nothing.
template <bool LDS, class C>
__device__ __forceinline__ void graze_pass(const DevScene& S, V3 o, V3 d, float& bt, uint32_t& bk, C& c,
                                           GrazePre pre, lfloat4* lnodes, bool novote = false) {
    if (S.n_graze_blk == 0) return;
    RT_T0(C, t_g);
    const float dd = len2(d);
    const float lim = S.graze_s2 * dd;
    if (S.graze_res) {
        const uint32_t* mp = S.graze_mask + (size_t)lb_cell(S.graze_res, d) * S.graze_words;
        cfloat4* tp = cptr(S.graze_tri);
        if (S.graze_lane) {
            lfloat4* lpn = lnodes + 4 * S.n_bvh_nodes;
            // the first two words requested together (one memory round trip where a scene has
            // at most 64 grazing pairs, config 3: 50)
            const uint32_t w0 = (false || novote) ? 0u : mp[0];
            const uint32_t w1 = (false || novote || S.graze_words < 2) ? 0u : mp[1];
            for (uint32_t w = 0; w < S.graze_words; ++w) {
                uint32_t own = novote ? 0u
                                      : (w == 0 ? (false ? pre.m0 : w0)
                                                : (w == 1 ? (false ? pre.m1 : w1) : mp[w]));
                RT_OPS(c, graze);
                uint32_t real = 0u;  // the pairs of word w this lane grazes
                while (own) {        // divergent: as many rounds as the longest list
                    const uint32_t b = (uint32_t)__builtin_ctz(own);
                    own &= own - 1u;
                    const uint32_t pi = 32u * w + b;
                    float4 a, e;
                    if (LDS) {
                        a = lpn[2 * pi];
                        e = lpn[2 * pi + 1];
                    } else {
                        a = S.graze_pn[2 * pi];
                        e = S.graze_pn[2 * pi + 1];
                    }
                    f2 nn = (bc(d.x) * f2{a.x, a.y} + bc(d.y) * f2{a.z, a.w}) + bc(d.z) * f2{e.x, e.y};
                    nn *= nn;
                    RT_OPS(c, graze_n);
                    if (nn.x < lim || nn.y < lim) real |= 1u << b;
                }
                uint32_t done = 0u;  // wave-uniform
                uint64_t pend;
                while ((pend = __ballot((real & ~done) != 0u)) != 0ull) {
                    uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)(real & ~done), (int)__builtin_ctzll(pend));
                    done |= m;
                    while (m) {
                        const uint32_t pi = 32u * w + (uint32_t)__builtin_ctz(m);
                        m &= m - 1u;
                        RT_OPS(c, tri);
                        tri_pair(ld_tri(tp + 6 * pi), o, d, bt, bk);
                    }
                }
            }
            RT_T1(C, c, cyc_graze, t_g);
            return;
        }
        cfloat4* pn = cptr(S.graze_pn);
        for (uint32_t w = 0; w < S.graze_words; ++w) {
            // the pairs this lane's direction cell lists: a superset of the pairs it grazes
            const uint32_t own = (false && w == 0) ? pre.m0 : ((false && w == 1) ? pre.m1 : mp[w]);
            RT_OPS(c, graze);
            // Every pair some active lane lists, each once: take the first lane that still
            // lists an untested pair, test all of its untested pairs, repeat.  Ballots and
            // readlane see exactly the active lanes, whatever they are (a butterfly of lane
            // shuffles can lose a lane's bits when the lane it passes through is inactive);
            // lanes of one direction cell share their list, so few rounds cover the wave.
            uint32_t done = 0u;  // wave-uniform
            uint64_t pend;
            while ((pend = __ballot((own & ~done) != 0u)) != 0ull) {
                uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)(own & ~done), (int)__builtin_ctzll(pend));
                done |= m;
                while (m) {
                    const uint32_t pi = 32u * w + (uint32_t)__builtin_ctz(m);
                    m &= m - 1u;
                    const float4 a = pn[2 * pi], b = pn[2 * pi + 1];
                    f2 nn = (bc(d.x) * f2{a.x, a.y} + bc(d.y) * f2{a.z, a.w}) + bc(d.z) * f2{b.x, b.y};
                    nn *= nn;
                    RT_OPS(c, graze_n);
                    if (__ballot(nn.x < lim || nn.y < lim)) {
                        RT_OPS(c, tri);
                        tri_pair(ld_tri(tp + 6 * pi), o, d, bt, bk);
                    }
                }
            }
        }
        RT_T1(C, c, cyc_graze, t_g);
        return;
    }
    cfloat4* g = cptr(S.graze_blk);
    cfloat4* tp = cptr(S.graze_tri);
    for (int b = 0; b < S.n_graze_blk; ++b, g += 8, tp += 24) {
        float4 a = g[0];
        float ca = (d.x * a.x + d.y * a.y) + d.z * a.z;
        RT_OPS(c, graze);
        if (!__ballot(ca * ca <= a.w * dd)) continue;
        RT_OPS(c, graze_n);
        float4 x0 = g[1], x1 = g[2], y0 = g[3], y1 = g[4], z0 = g[5], z1 = g[6];
        f2 n01 = (bc(d.x) * f2{x0.x, x0.y} + bc(d.y) * f2{y0.x, y0.y}) + bc(d.z) * f2{z0.x, z0.y};
        f2 n23 = (bc(d.x) * f2{x0.z, x0.w} + bc(d.y) * f2{y0.z, y0.w}) + bc(d.z) * f2{z0.z, z0.w};
        f2 n45 = (bc(d.x) * f2{x1.x, x1.y} + bc(d.y) * f2{y1.x, y1.y}) + bc(d.z) * f2{z1.x, z1.y};
        f2 n67 = (bc(d.x) * f2{x1.z, x1.w} + bc(d.y) * f2{y1.z, y1.w}) + bc(d.z) * f2{z1.z, z1.w};
        n01 *= n01;
        n23 *= n23;
        n45 *= n45;
        n67 *= n67;
        if (__ballot(n01.x < lim || n01.y < lim)) {
            RT_OPS(c, tri);
            tri_pair(ld_tri(tp), o, d, bt, bk);
        }
        if (__ballot(n23.x < lim || n23.y < lim)) {
            RT_OPS(c, tri);
            tri_pair(ld_tri(tp + 6), o, d, bt, bk);
        }
        if (__ballot(n45.x < lim || n45.y < lim)) {
            RT_OPS(c, tri);
            tri_pair(ld_tri(tp + 12), o, d, bt, bk);
        }
        if (__ballot(n67.x < lim || n67.y < lim)) {
            RT_OPS(c, tri);
            tri_pair(ld_tri(tp + 18), o, d, bt, bk);
        }
    }
    RT_T1(C, c, cyc_graze, t_g);
}

template <class C>
__device__ __forceinline__ void planes(const DevScene& S, V3 o, V3 d, float& bt, uint32_t& bk, C& c) {
    for (int i = 0; i < S.n_plane; ++i) {
        RT_OPS(c, plane);
        plane_one(cptr(S.plane) + 5 * i, o, d, bt, bk);
    }
}

// the primitives outside the hierarchy (all of them when it is off)
template <class C>
__device__ __forceinline__ void linear_rest(const DevScene& S, V3 o, V3 d, float& bt, uint32_t& bk, C& c) {
    run_dsph(S, S.n_dsph_bvh, S.n_dsph, o, d, bt, bk, c);
    run_gsph(S, S.n_gsph_bvh, S.n_gsph, o, d, bt, bk, c);
    run_tri(S, S.n_tri_bvh, S.n_tri, o, d, bt, bk, c);
    run_cube(S, S.n_cube_bvh, S.n_cube, o, d, bt, bk, c);
}

// Scene::intersect (scene/mod.rs:98-116): the nearest (t, key) over every shape, folded
// into the (t, key) the lane already holds (scan_from: bt / bk may hold a shape tested
// beforehand -- the lexicographic minimum does not depend on the order of the tests, and a
// smaller starting t only lets the walk cull more).
// LDS: the kernel staged the hierarchy's node records in LDS (lnodes).
template <bool LDS = false, class C>
__device__ __forceinline__ void scan_from(const DevScene& S, V3 o, V3 d, float& bt, uint32_t& bk, C& c,
                                          lfloat4* lnodes = nullptr) {
    RT_T0(C, t_s);
    RT_STAT(0);
    const GrazePre gp = graze_prefetch(S, d);
    planes(S, o, d, bt, bk, c);
    if (S.use_bvh) {
        bvh_walk<false, LDS>(S, o, d, bt, bk, 0.f, 0.f, c, lnodes);
        graze_pass<LDS>(S, o, d, bt, bk, c, gp, lnodes);
    }
    linear_rest(S, o, d, bt, bk, c);
    RT_T1(C, c, cyc_scan, t_s);
}
// scan_from for lanes that may hold a shape buffer (rt_build.cpp build_shape_buffers): a lane
// with buf_ok (its segment to the enclosing sphere's exit lies in the sphere's ball, bt = that
// exit) tests the buffer's records instead of walking the hierarchy; the wave takes its
// lanes' buffers one after the other, each tested like a leaf by every lane (a record tested
// for a lane that does not need it changes nothing), and walks the hierarchy for the other
// lanes only (buffered lanes do not vote).
template <bool LDS = false, class C>
__device__ __forceinline__ void scan_buffered(const DevScene& S, V3 o, V3 d, float& bt, uint32_t& bk, C& c,
                                              lfloat4* lnodes, bool buf_ok, uint32_t buf_leaf) {
    RT_T0(C, t_s);
    RT_STAT(0);
    const GrazePre gp = graze_prefetch(S, d);
    planes(S, o, d, bt, bk, c);
    if (S.use_bvh) {
        bool want = buf_ok;
        uint64_t pend;
        if ((pend = __ballot(want)) != 0) {
            const float on = sqrtf(len2(o));
            do {
                const uint32_t cur = (uint32_t)__builtin_amdgcn_readlane((int)buf_leaf, (int)__builtin_ctzll(pend));
                want = want && buf_leaf != cur;
                RT_T0(C, t_l);
                bvh_leaf(S, cur, o, d, on, bt, bt, bk, c);
                RT_T1(C, c, cyc_leaf, t_l);
            } while ((pend = __ballot(want)) != 0);
        }
        if (__ballot(!buf_ok)) bvh_walk<false, LDS>(S, o, d, bt, bk, 0.f, 0.f, c, lnodes, buf_ok);
        graze_pass<LDS>(S, o, d, bt, bk, c, gp, lnodes);
    }
    linear_rest(S, o, d, bt, bk, c);
    RT_T1(C, c, cyc_scan, t_s);
}

template <bool LDS = false, class C>
__device__ __forceinline__ void scan(const DevScene& S, V3 o, V3 d, float& bt, uint32_t& bk, C& c,
                                     lfloat4* lnodes = nullptr) {
    bt = __builtin_huge_valf();
    bk = 0xFFFFFFFFu;
    scan_from<LDS>(S, o, d, bt, bk, c, lnodes);
}

// ------------------------------------------------------------------ light buffers
// (rt_build.cpp build_light_buffers, DESIGN.md "Light buffers")

// max of x over the active lanes (NaN lanes ignored unless the first lane's is NaN, which
// only makes the caller's reach unbounded), wave-uniform: each round jumps to a lane above
// the current max.  Exact for any set of active lanes, and no LDS round trips (a butterfly
// of lane shuffles costs six and can lose a lane routed through an inactive one).
__device__ __forceinline__ float wave_max(float x) {
    float m = rfl(x);
    uint64_t b;
    while ((b = __ballot(x > m)) != 0ull) m = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), (int)__builtin_ctzll(b)));
    return m;
}

// The light-buffer pass of a shadow scan.  A lane with a buffer (lb) tests the records
// its cell lists; the wave takes its lanes' cells one after the other, each tested like
// a hierarchy leaf by every lane (a record tested for a lane whose cell does not list it
// changes nothing), until every lane is decided or done.  Afterwards an lb lane's
// hierarchy primitives are settled.
// A light-buffer cell: its runs, each nearest first, stopped at the first record whose
// nearest distance to the light exceeds `reach` (no undecided lane's origin is farther
// from the light, so nothing from there on can shadow one; the record's spare slot
// holds that distance).
// A cell's leaf record carries in bit 31 of its first run start whether its tier has an
// all-cell leaf (the records whose grown ball comes within LB_RHO of the light, listed once
// for the tier instead of in every cell): that leaf's runs follow the cell's.
template <class C>
__device__ __forceinline__ void lb_runs(const DevScene& S, uint4 a, uint4 b, V3 o, V3 d, float on, float tmax,
                                        float reach, float& bt, uint32_t& bk, C& c) {
    a.x &= 0x7FFFFFFFu;
    if (a.x < a.y) {
        cfloat4* p = cptr(S.dsph) + 4 * a.x;
        RT_PF_INIT(SphPair, ld_sph, p)
        for (uint32_t i = a.x; i < a.y; ++i) {
            RT_PF_NEXT(SphPair, ld_sph, p, 4)
            if (cur.q3.w > reach) break;
            RT_OPS(c, dsph);
            sph_pair(cur, o, d, bt, bk);
            RT_PF_ADV
        }
    }
    if (a.z < a.w) {
        cfloat4* p = cptr(S.gsph) + 4 * a.z;
        RT_PF_INIT(Rec16, ld_rec, p)
        for (uint32_t i = a.z; i < a.w; ++i) {
            RT_PF_NEXT(Rec16, ld_rec, p, 4)
            if (cur.rk.w > reach) break;
            RT_OPS(c, gsph);
            sph_general(cur, o, d, bt, bk);
            RT_PF_ADV
        }
    }
    if (b.x < b.y) {
        cfloat4* p = cptr(S.tri) + 6 * b.x;
        RT_PF_INIT(TriPair, ld_tri, p)
        for (uint32_t i = b.x; i < b.y; ++i) {
            RT_PF_NEXT(TriPair, ld_tri, p, 6)
            if (cur.q5.x > reach) break;
            RT_OPS(c, tri);
            tri_pair(cur, o, d, bt, bk);
            RT_PF_ADV
        }
    }
    if (b.z < b.w) {
        cfloat4* p = cptr(S.cube) + 4 * b.z;
        for (uint32_t i = b.z; i < b.w; ++i, p += 4) {
            const Rec16 r = ld_rec(p);
            if (r.rk.w > reach) break;
            cube_culled(r, o, d, on, tmax, bt, bk, c);
        }
    }
}
template <class C>
__device__ __forceinline__ void lb_leaf(const DevScene& S, uint32_t li, uint32_t all_li, V3 o, V3 d, float on,
                                        float tmax, float reach, float& bt, uint32_t& bk, C& c) {
    cuint4* lp = (cuint4*)S.bvh_leaves + 2 * li;
    const uint4 a = lp[0], b = lp[1];
    lb_runs(S, a, b, o, d, on, tmax, reach, bt, bk, c);
    if (a.x >> 31) {  // the tier's all-cell leaf
        cuint4* ap = (cuint4*)S.bvh_leaves + 2 * all_li;
        lb_runs(S, ap[0], ap[1], o, d, on, tmax, reach, bt, bk, c);
    }
}

// base: the lane's tier's first cell; all_leaf: that tier's all-cell leaf
template <class C>
__device__ __forceinline__ void lb_pass(const DevScene& S, uint32_t base, uint32_t all_leaf, V3 o, V3 d, float on,
                                        float tlim, float l2, bool lb, float& bt, uint32_t& bk, C& c) {
    const uint32_t leaf = lb ? base + lb_cell(S.lb_res, neg(d)) : 0u;
    bool want = lb && !shadow_decided(o, d, bt, l2);
    uint64_t pend;
    while ((pend = __ballot(want)) != 0) {
        const int owner = (int)__builtin_ctzll(pend);
        const uint32_t cur = (uint32_t)__builtin_amdgcn_readlane((int)leaf, owner);
        const uint32_t cur_all = (uint32_t)__builtin_amdgcn_readlane((int)all_leaf, owner);
        want = want && leaf != cur;
        RT_T0(C, t_l);
        const bool dec = shadow_decided(o, d, bt, l2);
        // the farthest undecided origin from the light (+ rounding margin) among the lanes
        // whose cell this is (the others test these records too, which changes nothing for
        // them: their own cell's complete list is their pass)
        const float reach = wave_max((dec || leaf != cur) ? 0.f : sqrtf(l2) * 1.001f + 1e-4f);
        lb_leaf(S, cur, cur_all, o, d, on, dec ? -1.f : fminf(bt, tlim), reach, bt, bk, c);  // decided lanes do not vote
        RT_T1(C, c, cyc_leaf, t_l);
        want = want && !shadow_decided(o, d, bt, l2);
    }
}

// Every hierarchy primitive for every lane, in leaf order: the shadow walk of a wave none of
// whose boxes can be culled (far origins: the box growth h(D) spans the scene ball), without
// the walk's node tests, stack and per-leaf dependent loads -- the records stream through the
// prefetching run loops.  Exact: a superset of what the walk tests (the nearest (t, key) does
// not depend on order or on extra records; a decided lane stays decided; a buffered lane's
// hierarchy primitives are settled, so extra records change nothing for it).  The grazing pass
// after it tests nothing new.  Stops when every lane is decided.  (Raising the wave's issue
// priority meanwhile -- such a task is the shadow pass's critical path -- measured flat.)
template <bool LDS, class C>
__device__ __forceinline__ void hier_linear(const DevScene& S, V3 o, V3 d, float& bt, uint32_t& bk, float tlim,
                                            float l2, C& c, lfloat4* lnodes) {
    constexpr int CH = 32;
    for (int b = 0; b < S.n_dsph_bvh; b += CH) {
        const int e = min(b + CH, S.n_dsph_bvh);
        if (LDS) run_dsph_lds(b, e, o, d, bt, bk, c, lds_dsph(S, lnodes));
        else run_dsph(S, b, e, o, d, bt, bk, c);
        if (__ballot(!shadow_decided(o, d, bt, l2)) == 0) return;
    }
    run_gsph(S, 0, S.n_gsph_bvh, o, d, bt, bk, c);
    run_tri(S, 0, S.n_tri_bvh, o, d, bt, bk, c);
    if (__ballot(!shadow_decided(o, d, bt, l2)) == 0) return;
    const float on = sqrtf(len2(o));
    cfloat4* p = cptr(S.cube);
    for (int i = 0; i < S.n_cube_bvh; ++i, p += 4) {
        const bool dec = shadow_decided(o, d, bt, l2);
        cube_culled(ld_rec(p), o, d, on, dec ? -1.f : fminf(bt, tlim), bt, bk, c);
    }
}

// ------------------------------------------------------------------ shadow scan
// PointLight::get_energy (scene/mod.rs:189-206): a FULL nearest-hit scan, then
// "shadowed iff |hit.point - p|^2 < |pos - p|^2".  Exact early exit:
//  * planes are scanned first; only planes can return t < 0 (plane.rs:62-83 has no
//    t >= 0 check; spheres and triangles reject t < 0), so after them a lane whose best
//    t is negative already holds its nearest hit;
//  * for t >= 0 the reference's distance |(p + d*t) - p|^2 is non-decreasing in t (each
//    rounded step is monotone), so once ANY hit has distance^2 < |pos - p|^2 the nearest
//    one does too;
//  * hits at t > tlim = ((1 + 2^-10) |pos - p| + 1e-5 (|p| + 1)) / |d| have a rounded
//    distance^2 >= |pos - p|^2 (the margin covers the rounding of p + d t and of the
//    norms) and can neither shadow nor hide a nearer hit: the walk stops at tlim.
// A wave leaves the scan when every active lane is decided.  Returns `shadowed`.
template <bool LDS, class C, bool SPLIT = false>
__device__ __forceinline__ bool shadow_scan(const DevScene& S, V3 o, V3 d, V3 lpos, C& c, lfloat4* lnodes,
                                            uint32_t lb_base = 0xFFFFFFFFu) {
    RT_T0(C, t_s);
    const GrazePre gp = graze_prefetch(S, d);
    const float l2 = len2(sub(lpos, o));
    float bt = __builtin_huge_valf();
    uint32_t bk = 0xFFFFFFFFu;
    // SPLIT (the shadow kernel's counting frames): planes in cyc_load, the light-buffer pass in
    // cyc_post, the hierarchy walk in cyc_self -- slots the trace kernel uses for other things
    RT_T0(C, t_pl);
    planes(S, o, d, bt, bk, c);
    if (SPLIT) RT_T1(C, c, cyc_load, t_pl);
    bool done = shadow_decided(o, d, bt, l2);
    if (__ballot(!done) == 0) goto finish;
    if (S.use_bvh) {
        float on = sqrtf(len2(o));
        float tlim = (sqrtf(l2) * (1.f + 0.0009765625f) + 1e-5f * (on + 1.f)) / sqrtf(len2(d));
        bool lb = false;
        if (S.lb_res) {
            const int tier = lb_tier(S, lb_base, o, l2);
            lb = tier >= 0;
            RT_T0(C, t_lb);
            if (__ballot(lb)) {
                // a light's leaves: its tiers' cells, then one all-cell leaf per tier
                const uint32_t nc = 6u * S.lb_res * S.lb_res, lb0 = lb_base & 0x0FFFFFFFu;
                const uint32_t tiers = (lb_base >> 28) & 7u;
                lb_pass(S, lb0 + (tier > 0 ? (uint32_t)tier * nc : 0u), lb0 + tiers * nc + (uint32_t)max(tier, 0), o, d,
                        on, tlim, l2, lb, bt, bk, c);
            }
            if (SPLIT) RT_T1(C, c, cyc_post, t_lb);
        }
        RT_T0(C, t_w);
#if RT_DIAG
        {  // slot 15: lanes a hierarchy walk serves (no light buffer, undecided); slots 16-21:
           // those lanes by D / R in (0,3] (3,6] (6,12] (12,25] (25,50] (50,inf); 22: light
           // farther than RT_LB_LMAX
            const bool w = !lb && !shadow_decided(o, d, bt, l2);
            const uint64_t wl = __ballot(w);
            const bool first = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) ==
                               (uint32_t)__builtin_ctzll(__ballot(1));
            if (wl && first) atomicAdd(&rt_scan_stats[15], (unsigned long long)__builtin_popcountll(wl));
            if (wl) {
                const float dx = o.x - S.bvh_cx, dy = o.y - S.bvh_cy, dz = o.z - S.bvh_cz;  // (stats)
                const float q = (sqrtf(dx * dx + dy * dy + dz * dz) + S.bvh_r) / S.bvh_r;
                const int b = q <= 3.f ? 0 : q <= 6.f ? 1 : q <= 12.f ? 2 : q <= 25.f ? 3 : q <= 50.f ? 4 : 5;
                for (int k = 0; k < 6; k++) {
                    const uint64_t m = __ballot(w && b == k);
                    if (m && first) atomicAdd(&rt_scan_stats[16 + k], (unsigned long long)__builtin_popcountll(m));
                }
                const uint64_t far_l = __ballot(w && l2 > RT_LB_LMAX * RT_LB_LMAX);
                if (far_l && first) atomicAdd(&rt_scan_stats[22], (unsigned long long)__builtin_popcountll(far_l));
            }
        }
#endif
        bool linear = false;
        {
            const bool walker = !lb && !shadow_decided(o, d, bt, l2);
            if (__ballot(walker)) {
                // the nearest walking origin's box growth (D = |o - c| + R as bvh_ray)
                const float dx = o.x - S.bvh_cx, dy = o.y - S.bvh_cy, dz = o.z - S.bvh_cz;
                const float D = sqrtf(dx * dx + dy * dy + dz * dz) + S.bvh_r;
                const float dmin = -wave_max(walker ? -D : -__builtin_huge_valf());
                linear = fmaf(fmaf(S.bvh_g2, dmin, S.bvh_g1), dmin, S.bvh_g0) >= S.walk_lin_h;
                if (linear) hier_linear<LDS>(S, o, d, bt, bk, tlim, l2, c, lnodes);
                else bvh_walk<true, LDS>(S, o, d, bt, bk, tlim, l2, c, lnodes, lb);
            }
        }
        if (SPLIT) RT_T1(C, c, cyc_self, t_w);
        done = shadow_decided(o, d, bt, l2);
        if (__ballot(!done) == 0) goto finish;
        if (!linear) graze_pass<LDS>(S, o, d, bt, bk, c, gp, lnodes, done);
        done = shadow_decided(o, d, bt, l2);
        if (__ballot(!done) == 0) goto finish;
    }
    linear_rest(S, o, d, bt, bk, c);
finish:
    RT_T1(C, c, cyc_scan, t_s);
    return shadow_hit(o, d, bt, l2);
}
