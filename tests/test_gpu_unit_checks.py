"""The scattering geometry's angle-free forms against the reference's angle forms, case by case.

k_event takes the incoming direction's azimuth as its cosine and sine (`azimuth_cs`), builds
the new direction by the angle-sum rule (`direction_cosine_cs`, ARTES.f90:1962-2052) and
decides the peel-off's rotation turn from sin(phi_old - phi_det) (`peel_rotation`,
4864-4920) -- no atan2 / acos.  The reference (restated below from ARTES.f90, as the oracle
does, oracle/artes_oracle.c:504-595, 725-746) works with the angles.  The two differ only by
rounding, and where a branch boundary (phi = 0 / pi, phi_old == phi_det, num = +-1) makes the
angle form jump, the quantity it selects is ~0 on both sides -- except the peel's half-turn
for a direction within ~1e-6 rad of vertical, where either form's decision is a rounding of
the other's (see the test).  These tests run the device
functions through the test-only library `libartes_unit.so` (artes_amd/csrc/unit_checks.hip)
on random cases and on cases placed exactly on those boundaries.
"""
import ctypes
import math
import os

import numpy as np
import pytest

LIB = os.path.join(os.path.dirname(__file__), "..", "artes_amd", "lib", "libartes_unit.so")
PI = math.pi

# the peel's interpolated matrix: Rayleigh-like with P34 != 0, so V is rotated too
SC = np.array([[1.0, -0.5, 0.0, 0.0], [-0.5, 1.0, 0.0, 0.0], [0.0, 0.0, 0.8, 0.3], [0.0, 0.0, -0.3, 0.8]])


def _lib():
    lib = ctypes.CDLL(LIB)
    f = lib.artes_unit_scatter_geometry
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p]
    f.restype = ctypes.c_int
    return f


def test_unit_library_exports():
    """CPU: the test library loads and exports its entry point (no device call)."""
    assert os.path.exists(LIB), "build with make -C artes_amd/csrc all"
    _lib()


# ---------------------------------------------------------------- the reference's forms
def _mueller(psi):
    """mueller_matrix_filler (ARTES.f90:1934-1960): (c2p, s2p) with its quadrant signs."""
    c2p = math.cos(2.0 * psi)
    s2p = math.sqrt(max(0.0, 1.0 - c2p * c2p))
    if (PI / 2 < psi < PI) or (3 * PI / 2 < psi < 2 * PI) or (-PI / 2 < psi < 0.0) or (-2 * PI < psi < -3 * PI / 2):
        s2p = -s2p
    return c2p, s2p


def _rotate(v, c, s):
    return [v[0], c * v[1] + s * v[2], -s * v[1] + c * v[2], v[3]]


def _renorm(out, ref):
    po = math.sqrt(out[1] ** 2 + out[2] ** 2 + out[3] ** 2)
    norm = math.sqrt(ref[1] ** 2 + ref[2] ** 2 + ref[3] ** 2) / po if po > 0 else 1.0
    if norm != 1.0:
        out[1] *= norm; out[2] *= norm; out[3] *= norm
    return out


def _polarization_rotation(alpha, beta, si, d2, dn2, errs):
    """polarization_rotation (ARTES.f90:1663-1932), the peeling branch (no renormalisation of I)."""
    if not (abs(alpha) < 1.0 and abs(dn2) < 1.0):
        errs.append(16)
        return [0.0] * 4
    num = (d2 - dn2 * alpha) / (math.sqrt(1.0 - alpha * alpha) * math.sqrt(1.0 - dn2 * dn2))
    beta2 = 0.0
    if abs(num) <= 1.0:
        beta2 = math.acos(num)
    elif 1.0 < num < 1.00001:
        beta2 = 0.0
    elif -1.00001 < num < -1.0:
        beta2 = PI
    else:
        errs.append(11)
    c, s = _mueller(beta)
    rot = _renorm(_rotate(si, c, s), si)
    q = [sum(SC[i, j] * rot[j] for j in range(4)) for i in range(4)]
    if 0.0 <= beta < PI:
        c, s = _mueller(beta2)
    elif PI <= beta < 2 * PI:
        c, s = _mueller(-beta2)
    else:
        c, s = 1.0, 0.0   # (the reference leaves m from mueller(beta); never reached here)
    return _renorm(_rotate(q, c, s), q)


def _peel(d, det, st, errs, turn=None):
    """peel_photon's rotation (ARTES.f90:4864-4920): (made, drop, Stokes).  `turn` (True /
    False) overrides the half-turn decision (the boundary cases, see the test)."""
    mu = d[0] * det[0] + d[1] * det[1] + d[2] * det[2]
    mu = 1.0 - 1e-10 if mu >= 1.0 else (-1.0 + 1e-10 if mu <= -1.0 else mu)
    phi_old = math.atan2(d[1], d[0])
    phi_old += 2 * PI if phi_old < 0 else 0.0
    phi_det = math.atan2(det[1], det[0])
    phi_det += 2 * PI if phi_det < 0 else 0.0
    if not abs(d[2]) < 1.0:
        errs.append(45)
        return False, False, [0.0] * 4
    num = (det[2] - d[2] * mu) / (math.sqrt(1.0 - mu * mu) * math.sqrt(1.0 - d[2] * d[2]))
    phs = 0.0
    if abs(num) < 1.0:
        phs = math.acos(num)
    elif num >= 1.0:
        phs = 1e-10
    elif num <= -1.0:
        phs = PI - 1e-10
    else:
        errs.append(44)
    turned = (0.0 <= phi_old - phi_det < PI) != (0.0 <= 2 * PI + phi_old - phi_det < PI)
    if turn is not None:
        turned = turn
    if turned:
        phs = 2 * PI - phs
    if phs < 0:
        phs += 2 * PI
    if not abs(mu) < 1.0:
        errs.append(49)
        return False, True, [0.0] * 4
    return True, False, _polarization_rotation(mu, phs, st, d[2], det[2], errs)


def _direction_cosine(alpha, beta, d, errs, clamp=None):
    """direction_cosine (ARTES.f90:1962-2052).  `clamp` (True / False) overrides whether num
    is clamped to +-(1 - 1e-10) (the boundary cases, see the test)."""
    cto = d[2] / math.sqrt(d[0] ** 2 + d[1] ** 2 + d[2] ** 2)
    sto = math.sqrt(1.0 - cto * cto)
    phi_old = math.atan2(d[1], d[0])
    phi_old += 2 * PI if phi_old < 0 else 0.0
    ctn = phi_new = 0.0
    if PI <= beta < 2 * PI:
        ctn = cto * alpha + sto * math.sqrt(1 - alpha * alpha) * math.cos(2 * PI - beta)
    elif 0 <= beta < PI:
        ctn = cto * alpha + sto * math.sqrt(1 - alpha * alpha) * math.cos(beta)
    else:
        errs.append(18)
    stn = math.sqrt(1.0 - ctn * ctn)
    num = (alpha - ctn * cto) / (stn * sto)
    if clamp is None:
        clamp = abs(num) >= 1.0
    if clamp:
        num = 1.0 - 1e-10 if num > 0 else -1.0 + 1e-10
    else:
        num = max(-1.0, min(1.0, num))
    if PI <= beta < 2 * PI:
        phi_new = phi_old - math.acos(num)
    elif 0 <= beta < PI:
        phi_new = phi_old + math.acos(num)
    else:
        errs.append(19)
    phi_new += 2 * PI if phi_new < 0 else 0.0
    phi_new -= 2 * PI if phi_new > 2 * PI else 0.0
    cpn = math.cos(phi_new)
    spn = math.sqrt(max(0.0, 1.0 - cpn * cpn)) * (1.0 if phi_new < PI else -1.0)
    return [stn * cpn, stn * spn, ctn]


def _num(alpha, beta, d):
    """direction_cosine's num before its clamps (ARTES.f90:1995-2005)."""
    cto = d[2] / math.sqrt(d[0] ** 2 + d[1] ** 2 + d[2] ** 2)
    sto = math.sqrt(1.0 - cto * cto)
    cb = math.cos(2 * PI - beta) if PI <= beta < 2 * PI else math.cos(beta)
    ctn = cto * alpha + sto * math.sqrt(1 - alpha * alpha) * cb
    return (alpha - ctn * cto) / (math.sqrt(1.0 - ctn * ctn) * sto)


# ---------------------------------------------------------------- cases
def _unit(v):
    v = np.asarray(v, dtype=np.float64)
    return v / np.linalg.norm(v)


def _cases(det_theta, det_phi, rng):
    """Incoming directions: random ones plus every boundary of the angle forms."""
    pd = math.atan2(math.sin(det_theta) * math.sin(det_phi), math.sin(det_theta) * math.cos(det_phi)) % (2 * PI)
    dirs = [_unit(v) for v in rng.normal(size=(400, 3))]
    for th in (0.3, 1.0, PI / 2, 2.5, 1e-6, PI - 1e-6):
        s, c = math.sin(th), math.cos(th)
        for ph in (0.0, PI, pd, (pd + PI) % (2 * PI), PI / 2, 3 * PI / 2, 2 * PI - 1e-15, 1e-15):
            dirs.append(np.array([s * math.cos(ph), s * math.sin(ph), c]))
        dirs.append(np.array([s, -0.0, c]))      # phi = -0: atan2 gives -0, azimuth_cs (1, -0)
        dirs.append(np.array([-s, -0.0, c]))     # phi = -pi
        dirs.append(np.array([-s, 0.0, c]))      # phi = pi
    out = []
    for d in dirs:
        for alpha, beta in ((rng.uniform(-1, 1), rng.uniform(0, 2 * PI)), (0.3, 0.0), (0.3, PI), (-0.7, 2 * PI - 1e-12),
                            (1 - 1e-12, 1.0), (-1 + 1e-12, 4.0), (0.5, PI - 1e-15)):
            q, u, v = rng.uniform(-0.5, 0.5, size=3)
            out.append([d[0], d[1], d[2], alpha, beta, 1.0, q, u, v])
    return np.array(out, dtype=np.float64)


@pytest.mark.gpu
@pytest.mark.parametrize("det_theta,det_phi", [(PI / 2, PI / 2), (PI / 2, 0.0), (PI / 2, PI), (0.7, 4.0), (2.2, 1e-9)])
def test_scatter_geometry_matches_angle_forms(det_theta, det_phi):
    f = _lib()
    rng = np.random.default_rng(int(det_theta * 1000 + det_phi * 10))
    cases = _cases(det_theta, det_phi, rng)
    n = len(cases)
    out = np.zeros((n, 8))
    err = np.zeros(64, dtype=np.uint64)
    sc = np.ascontiguousarray(SC.reshape(16))
    rc = f(cases.ctypes.data, n, det_theta, det_phi, sc.ctypes.data, out.ctypes.data, err.ctypes.data)
    assert rc == 0
    det = [math.sin(det_theta) * math.cos(det_phi), math.sin(det_theta) * math.sin(det_phi), math.cos(det_theta)]
    ref_errs = []
    worst_dir = worst_stokes = 0.0
    n_boundary = clamped = 0
    wd_case = ws_case = None
    for i in range(n):
        d = cases[i, :3]
        e = _direction_cosine(cases[i, 3], cases[i, 4], d, ref_errs)
        # A direction within ~1e-6 rad of vertical: 1 - dz^2 ~ 1e-12 carries a relative rounding
        # error ~1e-4 in the reference's (unfused) form and none in the device's fused one, so
        # sin(theta) and everything after it agree only to that conditioning there
        scale = 1e4 if abs(d[2]) > 1.0 - 1e-9 else 1.0
        dd = max(abs(a - b) for a, b in zip(e, out[i, :3]))
        # num = +-1 in exact arithmetic (beta = 0 or pi: the new direction in the old one's
        # meridian plane) is the clamp's boundary: the reference moves the azimuth by
        # acos(1 - 1e-10) = 1.4e-5 rad when num rounds to >= 1 and by ~1e-8 when it rounds below.
        # The device evaluates num as the reference does (no fused multiply-adds, correctly
        # rounded roots: device_common.hpp, direction_cosine_cs), so it must take the
        # reference's side there too: no either-side escape.
        if abs(abs(_num(cases[i, 3], cases[i, 4], d)) - 1.0) < 1e-9:
            n_boundary += 1
            clamped += abs(_num(cases[i, 3], cases[i, 4], d)) >= 1.0
        dd /= scale
        if dd > worst_dir:
            worst_dir, wd_case = dd, (list(cases[i]), e, list(out[i, :3]))
        made, drop, so = _peel(d, det, list(cases[i, 5:9]), ref_errs)
        flags = (1 if made else 0) + (2 if drop else 0)
        assert out[i, 7] == flags, (i, cases[i], out[i])
        if made:
            diff = max(abs(a - b) for a, b in zip(so, out[i, 3:7]))
            # On the half-turn's boundary (phi_old - phi_det within rounding of 0 or pi) either
            # decision is a rounding of the reference's: the vectors then lie in one plane with
            # z, where num = +-1 and both turns agree -- except for a direction within ~1e-6 of
            # vertical, whose num (through sqrt(1 - dz^2)) carries a relative error ~1e-4 in
            # both forms.  There the GPU must match the reference with one of the two turns.
            dphi = math.atan2(d[1], d[0]) - math.atan2(det[1], det[0])
            if abs(math.sin(dphi)) < 1e-9:
                other = _peel(d, det, list(cases[i, 5:9]), [], turn=True)[2], _peel(d, det, list(cases[i, 5:9]), [], turn=False)[2]
                diff = min(max(abs(a - b) for a, b in zip(o, out[i, 3:7])) for o in other)
            if diff / scale > worst_stokes:
                worst_stokes, ws_case = diff / scale, (list(cases[i]), so, list(out[i, 3:7]))
    # rounding only: ~1e-14 in general; the reference's own sqrt(1 - cos^2) near cos = +-1
    # (phi_new ~ 0 / pi, phs ~ 0 / pi) carries ~1e-8, and the 1e-10 clamps of num 5e-10
    # (near-vertical directions: scaled by their conditioning, above)
    assert worst_dir < 1e-7, (worst_dir, wd_case)
    assert n_boundary > 0 and clamped > 0, (n_boundary, clamped)   # (the clamp's side is exercised)
    assert worst_stokes < 1e-7, (worst_stokes, ws_case)
    for code in (44, 45, 49):
        assert int(err[code]) == ref_errs.count(code), (code, int(err[code]), ref_errs.count(code))
