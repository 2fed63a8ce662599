"""Pin the CPU oracle to the reference's own known-answer tests.

The reference (Rust) cannot be built here, so the oracle -- a C++
restatement of src/render.rs and its callees -- is pinned by restating every unit test
the reference holds for this path.  Each test cites the reference test it restates.
"""
import ctypes as C
import math

import numpy as np
import pytest

from oracle import oracle as O
from rust_tracer_amd import abi

EPS = np.float32(np.finfo(np.float32).eps)


def L():
    return O.lib()


def mat(fn, *args):
    out = (C.c_float * 16)()
    fn(*args, out)
    return np.array(out[:], np.float32).reshape(4, 4)


def fa(v):
    return O.farr(v)


def matmul(a, b):
    out = (C.c_float * 16)()
    L().oracle_matrix_mul(fa(a.ravel()), fa(b.ravel()), out)
    return np.array(out[:], np.float32).reshape(4, 4)


def inverse(a):
    out = (C.c_float * 16)()
    st = L().oracle_matrix_inverse(fa(a.ravel()), out)
    return st, np.array(out[:], np.float32).reshape(4, 4)


def scale(x, y, z):
    return mat(L().oracle_matrix_scale, x, y, z)


def translate(x, y, z):
    return mat(L().oracle_matrix_translate, x, y, z)


def rot(axis, deg):
    return mat(getattr(L(), "oracle_matrix_rotate_" + axis), deg)


IDENT = np.eye(4, dtype=np.float32)


# ---- src/math/matrix.rs tests (:314-532) -------------------------------------------

def test_matrix_creation_scalar_identity():  # matrix.rs:314-352
    assert np.array_equal(mat(L().oracle_matrix_identity), IDENT)


def test_matrix_transpose():  # matrix.rs:354-378
    t = (C.c_float * 16)()
    L().oracle_matrix_transpose(fa(scale(2, 3, 4).ravel()), t)
    assert np.array_equal(np.array(t[:], np.float32).reshape(4, 4), scale(2, 3, 4))
    tr = translate(1, 2, 3)
    L().oracle_matrix_transpose(fa(tr.ravel()), t)
    tt = np.array(t[:], np.float32).reshape(4, 4)
    assert not np.array_equal(tt, tr)
    for axis in "xyz":
        L().oracle_matrix_transpose(fa(rot(axis, 90).ravel()), t)
        rt = np.array(t[:], np.float32).reshape(4, 4)
        assert np.all(np.abs(rt - rot(axis, 270)) < EPS)  # rot(90)^T == rot(270)


def test_matrix_mul():  # matrix.rs:380-393
    assert np.all(np.abs(matmul(scale(2, 2, 2), IDENT) - scale(2, 2, 2)) < EPS)
    assert np.all(np.abs(matmul(scale(2, 2, 2), scale(2, 2, 2)) - scale(4, 4, 4)) < EPS)


def test_matrix_inverse():  # matrix.rs:395-429
    st, inv = inverse(scale(2, 3, 4))
    assert st == 0 and np.all(np.abs(matmul(scale(2, 3, 4), inv) - IDENT) < 2 * EPS)
    st, inv = inverse(IDENT)
    assert np.all(np.abs(inv - IDENT) < 2 * EPS)
    tr = translate(2, 2, -4)
    st, inv = inverse(tr)
    assert np.all(np.abs(matmul(inv, tr) - IDENT) < 2 * EPS)
    m = IDENT.copy()
    m[1][3] = 4
    st, inv = inverse(m)
    assert np.all(np.abs(matmul(inv, m) - IDENT) < 2 * EPS)
    rx = rot("x", 82)
    st, inv = inverse(rx)
    assert np.all(np.abs(matmul(rx, inv) - IDENT) < 2 * EPS)


def test_matrix_singular_is_an_error_not_a_panic():  # matrix.rs:116-117
    st, _ = inverse(np.zeros((4, 4), np.float32))
    assert st == 2  # RT_ERR_SINGULAR_MATRIX


def test_matrix_transformations():  # matrix.rs:431-457
    assert np.array_equal(scale(2, 3, 4), np.diag([2, 3, 4, 1]).astype(np.float32))
    t = translate(2, 3, 4)
    assert list(t[:3, 3]) == [2, 3, 4]


def _pt(fn, m, p):
    out = (C.c_float * 3)()
    fn(fa(m.ravel()), fa(p), out)
    return np.array(out[:], np.float32)


def _pt_r(fn, p, m):
    out = (C.c_float * 3)()
    fn(fa(p), fa(m.ravel()), out)
    return np.array(out[:], np.float32)


def test_point_and_vector_products():  # matrix.rs:497-532, point.rs:182-237, vector3.rs:253-303
    one = [1, 1, 1]
    assert list(_pt(L().oracle_matrix_pt_mul, scale(2, 3, 4), one)) == [2, 3, 4]
    assert list(_pt(L().oracle_matrix_pt_mul, translate(2, 3, 4), one)) == [3, 4, 5]
    assert list(_pt_r(L().oracle_pt_mat_mul, one, translate(2, 3, 4))) == [1, 1, 1]  # p*M ignores translation
    assert list(_pt(L().oracle_matrix_vec3_mul, translate(2, 3, 4), one)) == [1, 1, 1]
    assert list(_pt_r(L().oracle_vec3_mat_mul, one, scale(2, 3, 4))) == [2, 3, 4]
    want = {"x": ([1, -1, 1], [1, 1, -1]), "y": ([1, 1, -1], [-1, 1, 1]), "z": ([-1, 1, 1], [1, -1, 1])}
    for axis, (m_p, p_m) in want.items():
        assert np.all(np.abs(_pt(L().oracle_matrix_pt_mul, rot(axis, 90), one) - m_p) < EPS)
        assert np.all(np.abs(_pt_r(L().oracle_pt_mat_mul, one, rot(axis, 90)) - p_m) < EPS)
        assert np.all(np.abs(_pt(L().oracle_matrix_vec3_mul, rot(axis, 90), one) - m_p) < EPS)
        assert np.all(np.abs(_pt_r(L().oracle_vec3_mat_mul, one, rot(axis, 90)) - p_m) < EPS)


# ---- src/scene/sphere.rs tests (:178-218) ------------------------------------------

def sphere_hit(transform, o, d):
    h = O.oracle_hit()
    L().oracle_sphere_intersect(fa(np.asarray(transform, np.float32).ravel()), fa(o), fa(d), C.byref(h))
    return h


def test_sphere_intersection_no_transform():  # sphere.rs:178-196
    h = sphere_hit(IDENT, [0, 0, 2], [0, 0, -1])
    assert h.hit and h.t == 1.0
    assert not sphere_hit(IDENT, [0, 0, 2], [0, 1, 0]).hit
    h = sphere_hit(IDENT, [0, 1, 2], [0, 0, -1])
    assert h.hit and h.t == 2.0


def test_sphere_intersection_transform():  # sphere.rs:198-218
    tf = matmul(translate(0, 2, -2), scale(2, 2, 2))
    h = sphere_hit(tf, [0, 0, 2], [0, 0, -1])
    assert h.hit and h.t == 4.0
    assert not sphere_hit(tf, [0, 0, 2], [0, 1, 0]).hit
    h = sphere_hit(tf, [0, 2, 2], [0, 0, -1])
    assert h.hit and h.t == 2.0


# ---- src/scene/triangle.rs tests (:130-223) ----------------------------------------

def tri_normal(a, b, c):
    out = (C.c_float * 3)()
    L().oracle_triangle_normal(fa(a), fa(b), fa(c), out)
    return list(out[:])


def tri_hit(a, b, c, o, d):
    h = O.oracle_hit()
    L().oracle_triangle_intersect(fa(a), fa(b), fa(c), fa(o), fa(d), C.byref(h))
    return h


def test_triangle_creation():  # triangle.rs:130-149
    assert np.allclose(tri_normal([0, 0, 0], [1, 0, 0], [0, 1, 0]), [0, 0, 1], atol=EPS)
    assert np.allclose(tri_normal([1, 0, 0], [0, 0, 0], [0, 1, 0]), [0, 0, -1], atol=EPS)


def test_triangle_intersection():  # triangle.rs:152-173
    h = tri_hit([2, -2, 0], [-2, -2, 0], [-2, 2, 0], [0, 0, -4], [0, 0, 1])
    assert h.hit and h.t == 4.0
    assert np.allclose(h.point[:], [0, 0, 0], atol=EPS)
    assert np.allclose(h.normal[:], [0, 0, -1], atol=EPS)
    assert np.allclose(h.eye_dir[:], [0, 0, -1], atol=EPS)
    assert h.entering == 1


def test_triangle_behind_ray():  # triangle.rs:176-190
    assert not tri_hit([2, -2, 0], [-2, -2, 0], [-2, 2, 0], [0, 0, -4], [0, 0, -1]).hit


def test_triangle_shading_is_white():  # triangle.rs:193-223
    h = tri_hit([2, -1, 0], [-1, -1, 0], [-1, 2, 0], [0, 0, -4], [0, 0, 1])
    assert h.hit
    half = abi.rt_color(0.5, 0.5, 0.5)
    light = np.array([0, 0, -4], np.float32)
    p = np.array(h.point[:], np.float32)
    ldir = (light - p) / np.float32(np.sqrt(np.float32(np.dot(light - p, light - p))))
    out = abi.rt_color()
    L().oracle_phong_reflected_energy(C.byref(half), C.byref(half), C.byref(half), 60.0,
                                      C.byref(abi.rt_color(1, 1, 1)), fa(ldir), C.byref(h), C.byref(out))
    for c in (out.r, out.g, out.b):
        assert abs(c - 1.0) < EPS  # == WHITE under Color's epsilon equality


# ---- src/scene/plane.rs test (:122-130) --------------------------------------------

def test_plane_texture_axes():
    u, v = (C.c_float * 3)(), (C.c_float * 3)()
    L().oracle_plane_axes(fa([0, 1, 0]), u, v)
    assert float(np.dot(np.array(u[:]), [0, 1, 0])) == 0.0


# ---- src/scene/color.rs test (:192-211) --------------------------------------------

def test_color_checkerboard_and_quantise():
    out = abi.rt_color()
    L().oracle_checkerboard(0.5, 0.5, C.byref(out))  # same quadrant, u%2 == v%2 -> WHITE
    assert (out.r, out.g, out.b) == (1.0, 1.0, 1.0)
    L().oracle_checkerboard(1.5, 0.5, C.byref(out))
    assert out.r == 0.5
    L().oracle_checkerboard(-1.5, 0.5, C.byref(out))  # mixed signs: inverted parity
    assert out.r == 1.0
    rgb = np.array([[0.0, 1.0, 2.0, -1.0, np.nan, 0.99999]], np.float32)
    assert list(O.as_u8(rgb).ravel()) == [0, 255, 255, 0, 0, 254]  # saturating `as u8`


# ---- src/render_tree.rs test (:265-291) --------------------------------------------

def test_ray_forest_matches_basic_render_sizes():
    """RayTree::size semantics: a miss is 0 nodes; every hit adds one."""
    o = O.OracleScene()
    rgb, sizes = o.render_forest(32, 24, 1)
    _, cnt = o.render(32, 24, 1)
    assert sizes.max() <= 1
    assert int(sizes.sum()) == cnt["shadow_rays"] // 3  # one node per hit, 3 lights


def test_fresnel_opaque_is_one():
    """Opaque materials (ri = 0): r0 = ((1-0)/(1+0))^2 = 1 -> Schlick == 1."""
    f = L().oracle_fresnel_reflection(fa([0, 1, 0]), fa([0, 1, 0]), 1.0, 0.0)
    assert f == 1.0
