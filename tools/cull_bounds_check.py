"""Empirical check of the culling error bounds of rt_bvh (DESIGN.md "Exact culling").

The BVH may skip a primitive for a ray only if the reference's f32 test could not
report a hit there.  rt_bvh inflates every box by h(ray), a bound on how far the
point  X' = o + t' d  of a reported hit (t' = the f32 t the reference computes) can be
from the exact primitive.  This script replays the reference arithmetic in numpy
float32 (one rounding per operation, the reference's operation order: the same
expression trees as rt_scan.hpp / sphere.rs / triangle.rs / cube.rs) on adversarial
rays -- near-tangent to spheres, grazing cube faces and triangle planes, origins on
and far from the surface -- measures the exact (f64) distance of X' from the
primitive, and prints the largest ratio  distance / bound-basis  per primitive type.

  sphere   basis r_P * (7.5 eps (|l|^2 + 1) + eps (|l| + 1 + lam))
  cube     basis sigma_max(A) * eps * (|l| + 1 + lam)
  triangle basis eps * (|o - v0| + |e|max + |o| + |v0|) / (sin(alpha) * sin(phi))

with l = o' (the object-space origin), lam = |L|_F |o| + |s| (the magnitudes the
rounding of L o + s scales with), phi the angle between the ray and the triangle plane.

rt_build.cpp multiplies each basis by a safety factor that must exceed the ratios printed
here by a wide margin.  Triangles report two numbers: rho = distance / basis over rays
with sin(phi) < 0.1 (the grazing range, where 1/sin(phi) is large), and for steeper rays
distance * sin(alpha) / (eps (...)), i.e. rho / sin(phi) (the box growth rt_build.cpp
caps at TRI_STEEP).  The line distance of the ray from the triangle is printed for
reference only: the hierarchy bounds the reported POINT, which lies on the ray.

usage: python tools/cull_bounds_check.py [n_per_type=2000000] [seed=1]
"""
import sys

import numpy as np

F = np.float32
EPS = float(np.finfo(np.float32).eps)


def rand_rot(rng, n):
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    w, x, y, z = q.T
    return np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
        np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
        np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], 1)


def unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


# ---------------------------------------------------------------- f32 reference kernels
def pt_mul(L, s, p):  # ((p.x*r.x + p.y*r.y) + p.z*r.z) + r.w, per row
    return np.stack([((p[:, 0] * L[:, i, 0] + p[:, 1] * L[:, i, 1]) + p[:, 2] * L[:, i, 2]) + s[:, i]
                     for i in range(3)], -1)


def vec_mul(L, v):
    return np.stack([(v[:, 0] * L[:, i, 0] + v[:, 1] * L[:, i, 1]) + v[:, 2] * L[:, i, 2] for i in range(3)], -1)


def dot3(a, b):
    return (a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]) + a[:, 2] * b[:, 2]


def cross3(a, b):
    return np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1], a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2],
                     a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], -1)


def sphere_f32(to, td):
    """sphere.rs:58-97 + solve_quadratic :126-145 -> (hit, t)"""
    a = dot3(td, td)
    b = F(2) * dot3(td, to)
    c = dot3(to, to) - F(1)
    disc = b * b - (F(4) * a) * c
    hit = ~(disc < 0)
    with np.errstate(all="ignore"):
        small = np.abs(disc) < F(EPS)
        x = (F(-0.5) * b) / a
        sq = np.sqrt(np.maximum(disc, F(0)))
        q = np.where(b > 0, F(-0.5) * (b + sq), F(-0.5) * (b - sq))
        t0 = np.where(small, x, q / a)
        t1 = np.where(small, x, c / q)
    lo, hi = np.minimum(t0, t1), np.maximum(t0, t1)
    sw = t0 > t1
    t0, t1 = np.where(sw, t1, t0), np.where(sw, t0, t1)
    hit &= ~((t0 < 0) & (t1 < 0))
    t = np.where(t0 < 0, t1, t0)
    return hit, t


def mt_f32(o, d, v0, e1, e2):
    """triangle.rs:51-80 -> (hit, t)"""
    p = cross3(d, e2)
    det = dot3(e1, p)
    ok = ~(np.abs(det) < F(EPS))
    with np.errstate(all="ignore"):
        inv = F(1) / det
        tv = o - v0
        u = dot3(tv, p) * inv
        ok &= ~((u < 0) | (u > 1))
        q = cross3(tv, e1)
        v = dot3(d, q) * inv
        ok &= ~((v < 0) | (u + v > 1))
        t = dot3(e2, q) * inv
    ok &= ~(t < 0)
    return ok, t


# ---------------------------------------------------------------- exact geometry (f64)
def point_tri_dist(p, a, b, c):
    """distance from points p to triangles abc (all (n,3) f64)"""
    ab, ac = b - a, c - a
    n = np.cross(ab, ac)
    nn = np.sum(n * n, 1)
    w = p - a
    # barycentrics of the projection
    s = np.sum(np.cross(w, ac) * n, 1) / nn
    t = np.sum(np.cross(ab, w) * n, 1) / nn
    inside = (s >= 0) & (t >= 0) & (s + t <= 1)
    dplane = np.abs(np.sum(w * n, 1)) / np.sqrt(nn)

    def seg(p, x, y):
        e = y - x
        k = np.clip(np.sum((p - x) * e, 1) / np.sum(e * e, 1), 0, 1)
        return np.linalg.norm(p - (x + k[:, None] * e), axis=1)

    dedge = np.minimum(np.minimum(seg(p, a, b), seg(p, b, c)), seg(p, c, a))
    return np.where(inside, dplane, dedge)


def line_tri_dist(o, d, a, b, c):
    """distance from the infinite lines o + s d to triangles abc (f64)"""
    n = np.cross(b - a, c - a)
    dn = np.sum(d * n, 1)
    with np.errstate(all="ignore"):
        s = np.sum((a - o) * n, 1) / dn
    P = o + s[:, None] * d
    inside = np.isfinite(s) & (point_tri_dist(P, a, b, c) <= 1e-12 * (1 + np.linalg.norm(P, axis=1)))

    def line_seg(o, d, x, y):
        e = y - x
        w0 = o - x
        A, B, C = np.sum(d * d, 1), np.sum(d * e, 1), np.sum(e * e, 1)
        D, E = np.sum(d * w0, 1), np.sum(e * w0, 1)
        den = A * C - B * B
        with np.errstate(all="ignore"):
            k = np.where(den > 1e-300, (A * E - B * D) / den, 0.0)
        k = np.clip(k, 0, 1)
        q = x + k[:, None] * e                       # segment point; nearest line point to it
        t = np.sum((q - o) * d, 1) / A
        return np.linalg.norm(o + t[:, None] * d - q, axis=1)

    dd = np.minimum(np.minimum(line_seg(o, d, a, b), line_seg(o, d, b, c)), line_seg(o, d, c, a))
    return np.where(inside, 0.0, dd)


def report(name, ratio, extra=None):
    if ratio.size == 0:
        print(f"{name}: no reported hits")
        return 0.0
    m = float(np.max(ratio))
    print(f"{name}: {ratio.size} reported hits, max ratio {m:.3g}, p99.99 {np.quantile(ratio, 0.9999):.3g}")
    if extra:
        for k, v in extra.items():
            print(f"   {k}: {v}")
    return m


def check_spheres(rng, n):
    r = np.exp(rng.uniform(np.log(0.03), np.log(1.0), n))
    aniso = rng.random(n) < 0.5
    S = np.where(aniso[:, None], r[:, None] * np.exp(rng.uniform(-0.7, 0.7, (n, 3))), r[:, None])
    R = np.where(aniso[:, None, None], rand_rot(rng, n), np.eye(3)[None])
    A = R * S[:, None, :]                                    # world = A x + c
    c = rng.uniform(-5, 5, (n, 3))
    L64 = np.linalg.inv(A)
    L = L64.astype(F)
    s = (-np.einsum("nij,nj->ni", L64, c)).astype(F)
    Lx, sx = L.astype(np.float64), s.astype(np.float64)
    Ax = np.linalg.inv(Lx)
    cx = -np.einsum("nij,nj->ni", Ax, sx)
    rP = np.linalg.norm(Ax, ord=2, axis=(1, 2))
    # object-space origin at distance |l| (log-uniform, incl. just outside the surface)
    lmag = np.where(rng.random(n) < 0.2, 1 + np.exp(rng.uniform(np.log(1e-6), np.log(1e-2), n)),
                    np.exp(rng.uniform(np.log(1.02), np.log(2000.0), n)))
    lo = unit(rng.normal(size=(n, 3))) * lmag[:, None]
    # tangent point of a sphere of radius rho = 1 + delta
    delta = np.where(rng.random(n) < 0.7, np.sign(rng.normal(size=n)) * np.exp(rng.uniform(np.log(1e-9), np.log(0.1), n)),
                     rng.uniform(-1, 0.2, n))
    rho = np.minimum(1 + delta, lmag * 0.999)
    e = unit(np.cross(lo, rng.normal(size=(n, 3))))
    al = rho / lmag
    T = rho[:, None] * (al[:, None] * unit(lo) + np.sqrt(np.maximum(0, 1 - al * al))[:, None] * e)
    dobj = T - lo
    ow = np.einsum("nij,nj->ni", Ax, lo) + cx
    dw = unit(np.einsum("nij,nj->ni", Ax, dobj))
    o32, d32 = ow.astype(F), dw.astype(F)
    to, td = pt_mul(L, s, o32), vec_mul(L, d32)
    hit, t = sphere_f32(to, td)
    o64, d64 = o32.astype(np.float64)[hit], d32.astype(np.float64)[hit]
    X = o64 + t[hit].astype(np.float64)[:, None] * d64
    y = np.einsum("nij,nj->ni", Lx[hit], X) + sx[hit]
    need = rP[hit] * np.maximum(0, np.linalg.norm(y, axis=1) - 1)
    l = np.linalg.norm(np.einsum("nij,nj->ni", Lx[hit], o64) + sx[hit], axis=1)
    lam = np.linalg.norm(Lx[hit], axis=(1, 2)) * np.linalg.norm(o64, axis=1) + np.linalg.norm(sx[hit], axis=1)
    basis = rP[hit] * (7.5 * EPS * (l * l + 1) + EPS * (l + 1 + lam))
    return report("sphere", need / basis)


CUBE = [  # v0 signs (x0.5), e1, e2 -- rt_scan.hpp RT_CUBE_TRIS
    (1, -1, -1, -1, 0, 0, -1, 1, 0), (1, 1, -1, 0, -1, 0, -1, 0, 0), (1, -1, 1, -1, 1, 0, 0, 1, 0),
    (-1, 1, 1, 1, -1, 0, 0, -1, 0), (1, 1, -1, 0, 0, 1, 0, -1, 1), (1, -1, 1, 0, 0, -1, 0, 1, -1),
    (-1, 1, 1, 0, 0, -1, 0, -1, 0), (-1, -1, 1, 0, 1, -1, 0, 0, -1), (-1, 1, 1, 1, 0, 0, 1, 0, -1),
    (1, 1, -1, -1, 0, 0, -1, 0, 1), (1, -1, -1, 0, 0, 1, -1, 0, 1), (-1, -1, 1, 0, 0, -1, 1, 0, -1)]


def check_cubes(rng, n):
    S = np.exp(rng.uniform(np.log(0.05), np.log(2.0), (n, 3)))
    A = rand_rot(rng, n) * S[:, None, :]
    c = rng.uniform(-5, 5, (n, 3))
    L64 = np.linalg.inv(A)
    L = L64.astype(F)
    s = (-np.einsum("nij,nj->ni", L64, c)).astype(F)
    Lx, sx = L.astype(np.float64), s.astype(np.float64)
    Ax = np.linalg.inv(Lx)
    cx = -np.einsum("nij,nj->ni", Ax, sx)
    sig = np.linalg.norm(Ax, ord=2, axis=(1, 2))
    # object-space target near the surface: a face point, pushed off by a small amount
    face = rng.integers(0, 3, n)
    T = rng.uniform(-0.5, 0.5, (n, 3)) * np.where(rng.random((n, 1)) < 0.3, 1.0 + 1e-3 * rng.normal(size=(n, 1)), 1.0)
    T[np.arange(n), face] = np.sign(rng.normal(size=n)) * (0.5 + np.sign(rng.normal(size=n)) *
                                                          np.exp(rng.uniform(np.log(1e-9), np.log(1e-2), n)))
    # direction: random, often grazing the chosen face
    dobj = unit(rng.normal(size=(n, 3)))
    graze = rng.random(n) < 0.6
    comp = np.sign(rng.normal(size=n)) * np.exp(rng.uniform(np.log(1e-8), 0, n))
    dobj[graze, face[graze]] = comp[graze]
    dobj = unit(dobj)
    dist = np.exp(rng.uniform(np.log(1e-4), np.log(300.0), n))
    Tw = np.einsum("nij,nj->ni", Ax, T) + cx
    dw = unit(np.einsum("nij,nj->ni", Ax, dobj))
    ow = Tw - dist[:, None] * dw
    o32, d32 = ow.astype(F), dw.astype(F)
    to, td = pt_mul(L, s, o32), vec_mul(L, d32)
    best = np.full(n, np.inf, F)
    hit = np.zeros(n, bool)
    for (sx_, sy_, sz_, a, b, cc, dd, e, f) in CUBE:
        v0 = np.broadcast_to(np.array([0.5 * sx_, 0.5 * sy_, 0.5 * sz_], F), (n, 3))
        e1 = np.broadcast_to(np.array([a, b, cc], F), (n, 3))
        e2 = np.broadcast_to(np.array([dd, e, f], F), (n, 3))
        h, t = mt_f32(to, td, v0, e1, e2)
        take = h & (t < best)
        best = np.where(take, t, best)
        hit |= h
    o64, d64 = o32.astype(np.float64)[hit], d32.astype(np.float64)[hit]
    X = o64 + best[hit].astype(np.float64)[:, None] * d64
    y = np.einsum("nij,nj->ni", Lx[hit], X) + sx[hit]
    dobj_out = np.linalg.norm(np.maximum(np.abs(y) - 0.5, 0), axis=1)
    need = sig[hit] * dobj_out
    l = np.linalg.norm(np.einsum("nij,nj->ni", Lx[hit], o64) + sx[hit], axis=1)
    lam = np.linalg.norm(Lx[hit], axis=(1, 2)) * np.linalg.norm(o64, axis=1) + np.linalg.norm(sx[hit], axis=1)
    basis = sig[hit] * EPS * (l + 1 + lam)
    return report("cube", need / basis)


def check_triangles(rng, n, phi_lo=1e-7, phi_hi=np.pi / 2, detail=False):
    v0 = rng.uniform(-4, 4, (n, 3))
    size = np.exp(rng.uniform(np.log(0.05), np.log(3.0), n))
    e1 = unit(rng.normal(size=(n, 3))) * size[:, None] * rng.uniform(0.3, 1, (n, 1))
    e2 = unit(rng.normal(size=(n, 3))) * size[:, None] * rng.uniform(0.3, 1, (n, 1))
    v1, v2 = v0 + e1, v0 + e2
    V0, V1, V2 = v0.astype(F), v1.astype(F), v2.astype(F)
    E1, E2 = V1 - V0, V2 - V0                                    # triangle.rs:52-53, f32
    a, b, cc = (x.astype(np.float64) for x in (V0, V1, V2))
    N = np.cross(b - a, cc - a)
    Nn = unit(N)
    sin_a = np.linalg.norm(N, axis=1) / (np.linalg.norm(b - a, axis=1) * np.linalg.norm(cc - a, axis=1))
    # target near the triangle (barycentric, slightly outside sometimes)
    u = rng.uniform(-0.05, 1.0, n)
    v = rng.uniform(-0.05, 1.0, n) * (1 - np.clip(u, 0, 1))
    T = a + u[:, None] * (b - a) + v[:, None] * (cc - a)
    T += Nn * (np.sign(rng.normal(size=n)) * np.exp(rng.uniform(np.log(1e-9), np.log(1e-1), n)))[:, None]
    # direction at angle phi to the plane
    phi = np.exp(rng.uniform(np.log(phi_lo), np.log(phi_hi), n))
    inpl = unit(np.cross(Nn, rng.normal(size=(n, 3))))
    d = unit(np.cos(phi)[:, None] * inpl + (np.sin(phi) * np.sign(rng.normal(size=n)))[:, None] * Nn)
    dist = np.exp(rng.uniform(np.log(1e-3), np.log(60.0), n))
    o = T - dist[:, None] * d
    o32, d32 = o.astype(F), d.astype(F)
    hit, t = mt_f32(o32, d32, V0, E1, E2)
    o64, d64 = o32.astype(np.float64)[hit], d32.astype(np.float64)[hit]
    X = o64 + t[hit].astype(np.float64)[:, None] * d64
    need = point_tri_dist(X, a[hit], b[hit], cc[hit])
    sphi = np.abs(np.sum(d64 * Nn[hit], 1)) / np.linalg.norm(d64, axis=1)
    emax = np.maximum(np.linalg.norm(b - a, axis=1), np.linalg.norm(cc - a, axis=1))[hit]
    tv = np.linalg.norm(o64 - a[hit], axis=1)
    basis = EPS * (tv + emax + np.linalg.norm(o64, axis=1) + np.linalg.norm(a[hit], axis=1)) / (
        sin_a[hit] * np.maximum(sphi, 1e-30))
    ratio = need / basis
    lat = line_tri_dist(o64, d64, a[hit], b[hit], cc[hit])
    lbasis = EPS * (tv + emax + np.linalg.norm(o64, axis=1) + np.linalg.norm(a[hit], axis=1)) / sin_a[hit]
    lratio = lat / lbasis
    buckets = {"LATERAL (line distance, no 1/sin(phi))": f"max ratio {lratio.max():.3g}"}
    for lo_, hi_ in ((1e-8, 1e-5), (1e-5, 1e-4), (1e-4, 3e-4), (3e-4, 1e-3), (1e-3, 2e-3), (2e-3, 1e-2),
                     (1e-2, 1e-1), (1e-1, 1.01)):
        m = (sphi >= lo_) & (sphi < hi_)
        if m.any():
            buckets[f"sin(phi) in [{lo_:g},{hi_:g})"] = (f"n={m.sum()} max ratio {ratio[m].max():.3g}, "
                                                         f"lateral {lratio[m].max():.3g}")
    if detail:
        return dict(lratio=lratio, ratio=ratio, sphi=sphi, sin_a=sin_a[hit], o=o64, d=d64, v=(a[hit], b[hit], cc[hit]),
                    t=t[hit], lat=lat, lbasis=lbasis, dist=dist[hit], V=(V0[hit], V1[hit], V2[hit]), o32=o32[hit], d32=d32[hit])
    small = sphi < 0.1
    rho_small = float(ratio[small].max()) if small.any() else 0.0
    steep = float((ratio / np.maximum(sphi, 1e-30))[~small].max()) if (~small).any() else 0.0
    report("triangle", ratio, buckets)
    return rho_small, steep


def run(n, seed, chunk=500000):
    """largest measured ratio per primitive type over n adversarial rays each"""
    rng = np.random.default_rng(seed)
    worst = {"sphere": 0.0, "cube": 0.0, "triangle": 0.0, "triangle_steep": 0.0}
    for k in range(0, n, chunk):
        m = min(chunk, n - k)
        worst["sphere"] = max(worst["sphere"], check_spheres(rng, m))
        worst["cube"] = max(worst["cube"], check_cubes(rng, m))
        tri, steep = check_triangles(rng, m)
        worst["triangle"] = max(worst["triangle"], tri)
        worst["triangle_steep"] = max(worst["triangle_steep"], steep)
    return worst


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000000
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    print("WORST", run(n, seed))


if __name__ == "__main__":
    main()
