// transport.hip -- MI355X (gfx950) photon-packet transport engine + C ABI.
//
// The hot path of the reference, `radiative_transfer` (ARTES.f90:518-1006), runs here
// as ONE persistent HIP kernel: one packet per lane, 64-lane waves, each lane
// refilling itself with the next packet of its static interleaved share as soon as
// its packet ends.  A packet's life is a state machine whose dominant state is a
// single uniform "trace step" (one cell_face call, ARTES.f90:2800-3470), shared by
// the three traces of the reference -- first optical depth (625-656), propagation
// (689-778 / 848-941) and peel-off (4739-4761) -- so the branchy geometry runs
// converged across the wave.  The rare, expensive event (peel contribution +
// scattering, ~2.5 per packet vs ~110 trace steps) is deferred until enough lanes of
// the wave need it (`R.defer`), so it runs with many lanes active instead of
// executing almost every iteration with one or two.
//
// All arithmetic is FP64 (the reference is double precision; the cell-face
// quadratics cancel ~15 digits at R ~ 7e7 m).  Tables: see tables.hpp.
// Detector: FP64 atomics into NCOPY privatised copies (copy = blockIdx % NCOPY, i.e.
// one per XCD under round-robin dispatch -- a speed heuristic only), summed by a
// small reduce kernel.  No MFMA: this is branchy per-packet work, not a contraction.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>

#include "tables.hpp"

namespace artes {

constexpr int NCOPY = 8;
constexpr int BLOCK = 256;
constexpr double PI = 3.14159265358979323846;
constexpr double HALF_PI = PI / 2.0;
constexpr double TWO_PI = 2.0 * PI;

// -------------------------------------------------------------- device data ---
struct DevGrid {
    int nr, ntheta, nphi, ncell;
    int cell_depth;
    double ax2, by2, cz2, a, b;
    double rtop;
    const double* __restrict__ rf2;      // [nr+1]
    const double* __restrict__ thetaf;   // [ntheta+1]
    const double* __restrict__ tan2;     // [ntheta+1]
    const int* __restrict__ tplane;      // [ntheta+1]
    const double* __restrict__ phif;     // [nphi]
    const double* __restrict__ phis;     // [nphi]
    const double* __restrict__ phic;     // [nphi]
    const double* __restrict__ kappa;    // [ncell] (this wavelength)
    const double* __restrict__ albedo;   // [ncell]
    const int* __restrict__ matid;       // [ncell]
    const double* __restrict__ mats;     // [nmat][180][16]
    const double* __restrict__ cums;     // [nmat][181][4]
    const double* __restrict__ sc2;      // [181]
    const double* __restrict__ ss2;      // [181]
};

struct DevRun {
    uint64_t first, n, seed;
    int nx, ny, photon_scattering, phase_far, stellar_direction, defer;
    double det0, det1, det2, sdt, cdt, sdp, cdp;
    double x_max, y_max, fstop, pmin, surface_albedo, theta_star, phi_star;
    double* __restrict__ det;       // [NCOPY][4][4][ny][nx]
    size_t det_stride;              // doubles per copy
    double* __restrict__ tot2;      // [4] packet-level sum T^2 per Stokes
    unsigned long long* __restrict__ cnt;   // [ARTES_NUM_COUNTERS]
    unsigned long long* __restrict__ err;   // [ARTES_NUM_ERR]
    double* __restrict__ rec;       // [n][4] (TRACE builds)
};

// ------------------------------------------------------------------- RNG ---
// One xoroshiro128++ stream per global packet id; identical to oracle/artes_oracle.c.
__device__ __forceinline__ uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
struct Rng {
    uint64_t s0, s1;
    __device__ __forceinline__ void seed(uint64_t seed, uint64_t id) {
        uint64_t k = seed;
        uint64_t sm = splitmix64(k) + 2ULL * id * 0x9e3779b97f4a7c15ULL;
        s0 = splitmix64(sm);
        s1 = splitmix64(sm);
        if ((s0 | s1) == 0) s1 = 1;
    }
    __device__ __forceinline__ double uni() {
        const uint64_t a = s0;
        uint64_t b = s1;
        const uint64_t res = rotl64(a + b, 17) + a;
        b ^= a;
        s0 = rotl64(a, 49) ^ b ^ (b << 21);
        s1 = rotl64(b, 28);
        return ((double)(res >> 11) + 0.5) * 0x1.0p-53;
    }
};

__device__ __forceinline__ void log_err(const DevRun& R, int code) { atomicAdd(&R.err[code], 1ULL); }

// sin/cos for |x| <~ 1e5 (every angle here is < 4 pi): two-constant Cody-Waite reduction
// by pi/2 with FMA, fdlibm __kernel_sin/__kernel_cos minimax polynomials on [-pi/4, pi/4].
// Absolute error ~1e-16; avoids the Payne-Hanek path (and its registers) of ocml cos/sin.
__device__ __forceinline__ void sincos_bounded(double x, double& s, double& c) {
    const double n = rint(x * 0.63661977236758134308);
    double r = fma(-n, 1.57079632679489655800e+00, x);
    r = fma(-n, 6.12323399573676603587e-17, r);
    const double z = r * r;
    const double ps = z * (8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 + z * (2.75573137070700676789e-06 +
                      z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10))));
    const double sr = r + r * z * (-1.66666666666666324348e-01 + ps);
    const double pc = z * z * (4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 + z * (2.48015872894767294178e-05 +
                      z * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + pc);
    const int q = ((int)n) & 3;
    s = (q == 0) ? sr : (q == 1) ? cr : (q == 2) ? -sr : -cr;
    c = (q == 0) ? cr : (q == 1) ? -sr : (q == 2) ? -cr : sr;
}
__device__ __forceinline__ double cos_b(double x) { double s, c; sincos_bounded(x, s, c); return c; }
__device__ __forceinline__ double sin_b(double x) { double s, c; sincos_bounded(x, s, c); return s; }

// ------------------------------------------------------------- geometry ---
// quadratic_equation (ARTES.f90:4154-4173)
__device__ __forceinline__ void quad_roots(double a, double b, double c, double& s0, double& s1) {
    s0 = 0.0;
    s1 = 0.0;
    const double disc = b * b - 4.0 * a * c;
    if (disc >= 0.0) {
        const double q = -0.5 * (b + copysign(sqrt(disc), b));
        if (fabs(a) > 1.e-100) s0 = q / a;
        if (fabs(q) > 1.e-100) s1 = c / q;
    }
}
// root selection block of cell_face (e.g. ARTES.f90:2897-2907)
__device__ __forceinline__ double pick_root(double s0, double s1, double tol) {
    if (s0 > tol && s1 <= tol && s0 < 1.e100) return s0;
    if (s1 > tol && s0 <= tol && s1 < 1.e100) return s1;
    if (s0 > tol && s1 > tol) {
        if (s0 < 1.e100 && s0 < s1) return s0;
        if (s1 < 1.e100 && s1 < s0) return s1;
    }
    return 0.0;
}

// theta cone x^2+y^2 = z^2 tan^2(theta_f) with the nappe filter (ARTES.f90:3026-3064)
__device__ __forceinline__ double cone_distance(const DevGrid& G, int f, double x, double y, double z,
                                                double n0, double n1, double n2, double tol) {
    const double t2 = G.tan2[f];
    const double qa = G.ax2 * n0 * n0 + G.by2 * n1 * n1 - G.cz2 * n2 * n2 * t2;
    const double qb = 2.0 * (G.ax2 * x * n0 + G.by2 * y * n1 - G.cz2 * z * n2 * t2);
    const double qc = G.ax2 * x * x + G.by2 * y * y - G.cz2 * z * z * t2;
    double s0, s1;
    quad_roots(qa, qb, qc, s0, s1);
    const double th = G.thetaf[f];
    if (s0 > 1.e-15) {
        const double zt = z + s0 * n2;
        if ((zt > 0.0 && th > HALF_PI) || (zt < 0.0 && th < HALF_PI)) s0 = 0.0;
    }
    if (s1 > 1.e-15) {
        const double zt = z + s1 * n2;
        if ((zt > 0.0 && th > HALF_PI) || (zt < 0.0 && th < HALF_PI)) s1 = 0.0;
    }
    return pick_root(s0, s1, tol);
}

struct Step {
    double d;
    int nft, nfi, ncr, nct, ncp;
    bool exit, err;
};

// cell_face + next_cell (ARTES.f90:2671-3470) in a uniform form: every cell has an
// inner and an outer face per coordinate; "same face" re-crossings of the face the
// packet sits on use the reference's 1e-3 tolerance in the matching slot.  The
// candidate set, tolerances and two-pass (>1e-9, then >1e-12) selection are the
// reference's; DESIGN.md §3 walks through the equivalence.
template <bool G3D>
__device__ __forceinline__ void cell_face(const DevGrid& G, const DevRun& R, double x, double y, double z,
                                          double n0, double n1, double n2, int ft, int fi, int cr, int ct, int cp,
                                          Step& o) {
    const double qa = G.ax2 * n0 * n0 + G.by2 * n1 * n1 + G.cz2 * n2 * n2;
    const double qb = 2.0 * (G.ax2 * x * n0 + G.by2 * y * n1 + G.cz2 * z * n2);
    const double S = G.ax2 * x * x + G.by2 * y * y + G.cz2 * z * z;
    double s0, s1;
    double d_rin = 0.0, d_rout = 0.0;
    if (!(ft == 1 && fi == cr)) {                      // inner sphere r_cell
        quad_roots(qa, qb, S - G.rf2[cr], s0, s1);
        d_rin = pick_root(s0, s1, 1.e-15);
    }
    {                                                  // outer sphere r_cell+1 (same face: 1e-3)
        quad_roots(qa, qb, S - G.rf2[cr + 1], s0, s1);
        d_rout = pick_root(s0, s1, (ft == 1 && fi == cr + 1) ? 1.e-3 : 1.e-15);
    }
    double d_tin = 0.0, d_tout = 0.0, d_pin = 0.0, d_pout = 0.0;
    int pout = 0;
    if constexpr (G3D) {
        const bool on_t = (ft == 2);
        if (ct != 0) {                                 // inner theta face (index ct)
            if (on_t && fi == ct) {
                if (G.thetaf[ct] > HALF_PI && G.tplane[ct] == 1) d_tin = cone_distance(G, ct, x, y, z, n0, n1, n2, 1.e-3);
            } else if (G.tplane[ct] == 1) {
                d_tin = cone_distance(G, ct, x, y, z, n0, n1, n2, 1.e-15);
            } else {
                if (-z / n2 > 0.0 && n2 > 1.e-15) d_tin = -z / n2;
            }
        }
        if (ct + 1 != G.ntheta) {                      // outer theta face (index ct+1)
            if (on_t && fi == ct + 1) {
                if (G.thetaf[ct + 1] < HALF_PI && G.tplane[ct + 1] == 1) d_tout = cone_distance(G, ct + 1, x, y, z, n0, n1, n2, 1.e-3);
            } else if (G.tplane[ct + 1] == 1) {
                d_tout = cone_distance(G, ct + 1, x, y, z, n0, n1, n2, 1.e-15);
            } else {
                if (-z / n2 > 0.0 && n2 < -1.e-15) d_tout = -z / n2;
            }
        }
        if (G.nphi > 1) {                              // phi half-planes (ARTES.f90:3292-3350)
            pout = (cp + 1 == G.nphi) ? 0 : cp + 1;
            const bool on_p = (ft == 3);
            double sp0 = 0.0;
            if (!(on_p && fi == cp)) {
                const double den = G.b * n1 * G.phic[cp] - G.a * n0 * G.phis[cp];
                if (fabs(den) > 0.0) {
                    sp0 = (G.a * x * G.phis[cp] - G.b * y * G.phic[cp]) / den;
                    if (sp0 > 1.e-15 && sp0 < 1.e100) d_pin = sp0;
                }
            }
            if (!(on_p && fi == pout)) {
                const double den = G.b * n1 * G.phic[pout] - G.a * n0 * G.phis[pout];
                if (fabs(den) > 0.0) {
                    const double sp1 = (G.a * x * G.phis[pout] - G.b * y * G.phic[pout]) / den;
                    if (sp1 > 1.e-15 && sp0 < 1.e100) d_pout = sp1;   // sic: sp0 (ARTES.f90:3318, 3346)
                }
            }
        }
    }
    // nearest face, 'large' then 'small' solutions (ARTES.f90:3358-3418)
    double best = 1.e100;
    int which = -1;
#define ARTES_CONSIDER(dd, w, thr) if ((dd) > (thr) && (dd) < best) { best = (dd); which = (w); }
    ARTES_CONSIDER(d_rin, 0, 1.e-9)
    if constexpr (G3D) { ARTES_CONSIDER(d_tin, 1, 1.e-9) ARTES_CONSIDER(d_pin, 2, 1.e-9) }
    ARTES_CONSIDER(d_rout, 3, 1.e-9)
    if constexpr (G3D) { ARTES_CONSIDER(d_tout, 4, 1.e-9) ARTES_CONSIDER(d_pout, 5, 1.e-9) }
    if (which < 0) {
        best = 1.e100;
        ARTES_CONSIDER(d_rin, 0, 1.e-12)
        if constexpr (G3D) { ARTES_CONSIDER(d_tin, 1, 1.e-12) ARTES_CONSIDER(d_pin, 2, 1.e-12) }
        ARTES_CONSIDER(d_rout, 3, 1.e-12)
        if constexpr (G3D) { ARTES_CONSIDER(d_tout, 4, 1.e-12) ARTES_CONSIDER(d_pout, 5, 1.e-12) }
    }
#undef ARTES_CONSIDER
    o.d = best;
    o.ncr = cr; o.nct = ct; o.ncp = cp;
    o.err = false;
    switch (which) {
        case 0: o.nft = 1; o.nfi = cr; o.ncr = cr - 1; break;
        case 3: o.nft = 1; o.nfi = cr + 1; o.ncr = cr + 1; break;
        case 1: o.nft = 2; o.nfi = ct; o.nct = ct - 1; break;
        case 4: o.nft = 2; o.nfi = ct + 1; o.nct = ct + 1; break;
        case 2: o.nft = 3; o.nfi = cp; o.ncp = (cp == 0) ? G.nphi - 1 : cp - 1; break;
        case 5: o.nft = 3; o.nfi = pout; o.ncp = pout; break;
        default: o.nft = 0; o.nfi = -999; o.err = true; log_err(R, 31); break;
    }
    o.exit = (o.nft == 1 && o.nfi == G.nr);
    if (ft == 1 && fi == G.cell_depth && o.nft == 1 && o.nfi == G.cell_depth) { o.err = true; log_err(R, 34); }
    if (o.ncr < 0) o.ncr = 0;
}

// ---------------------------------------------------- scattering physics ---
// mueller_matrix_filler (ARTES.f90:1934-1960): returns c2p, s2p
__device__ __forceinline__ void mueller(double psi, double& c2p, double& s2p) {
    c2p = cos_b(2.0 * psi);
    s2p = sqrt(1.0 - c2p * c2p);
    if ((psi > HALF_PI && psi < PI) || (psi > 1.5 * PI && psi < TWO_PI) || (psi > -HALF_PI && psi < 0.0) ||
        (psi > -TWO_PI && psi < -1.5 * PI))
        s2p = -s2p;
}

// polarization_rotation (ARTES.f90:1663-1932); sc is scatter(4,4) row-major
__device__ void polarization_rotation(const DevRun& R, double alpha, double beta, const double si[4],
                                      const double sc[16], double d2, double dn2, double so[4], bool peeling) {
    if (fabs(alpha) < 1.0 && fabs(dn2) < 1.0) {
        double beta2 = 0.0;
        const double num = (d2 - dn2 * alpha) / (sqrt(1.0 - alpha * alpha) * sqrt(1.0 - dn2 * dn2));
        if (fabs(num) <= 1.0) beta2 = acos(num);
        else if (num > 1.0 && num < 1.00001) beta2 = 0.0;
        else if (num < -1.0 && num > -1.00001) beta2 = PI;
        else log_err(R, 11);
        double c, s;
        mueller(beta, c, s);
        double r0 = si[0], r1 = c * si[1] + s * si[2], r2 = -s * si[1] + c * si[2], r3 = si[3];
        const double pr = sqrt(r1 * r1 + r2 * r2 + r3 * r3);
        double norm = (pr > 0.0) ? sqrt(si[1] * si[1] + si[2] * si[2] + si[3] * si[3]) / pr : 1.0;
        if (norm < 1.0 || norm > 1.0) { r1 *= norm; r2 *= norm; r3 *= norm; }
        double q[4];
#pragma unroll
        for (int i = 0; i < 4; i++) q[i] = sc[i * 4 + 0] * r0 + sc[i * 4 + 1] * r1 + sc[i * 4 + 2] * r2 + sc[i * 4 + 3] * r3;
        if (!peeling) {
            if (q[0] > 0.0) {
                norm = r0 / q[0];
#pragma unroll
                for (int i = 0; i < 4; i++) q[i] *= norm;
            } else {
                log_err(R, 12);
            }
        }
        if (beta >= 0.0 && beta < PI) mueller(beta2, c, s);
        else if (beta >= PI && beta < TWO_PI) mueller(-beta2, c, s);
        so[0] = q[0];
        so[1] = c * q[1] + s * q[2];
        so[2] = -s * q[1] + c * q[2];
        so[3] = q[3];
        const double po = sqrt(so[1] * so[1] + so[2] * so[2] + so[3] * so[3]);
        norm = (po > 0.0) ? sqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]) / po : 1.0;
        if (norm < 1.0 || norm > 1.0) { so[1] *= norm; so[2] *= norm; so[3] *= norm; }
    } else if (alpha >= 1.0 && alpha < 1.0001) {
#pragma unroll
        for (int i = 0; i < 4; i++) so[i] = si[i];
        log_err(R, 13);
    } else if (alpha <= -1.0 && alpha > -1.0001) {
        double q[4];
#pragma unroll
        for (int i = 0; i < 4; i++) q[i] = sc[i * 4 + 0] * si[0] + sc[i * 4 + 1] * si[1] + sc[i * 4 + 2] * si[2] + sc[i * 4 + 3] * si[3];
        if (peeling) {
            for (int i = 0; i < 4; i++) so[i] = q[i];
        } else if (q[0] > 0.0) {
            const double norm = si[0] / q[0];
            for (int i = 0; i < 4; i++) so[i] = norm * q[i];
        } else {
            for (int i = 0; i < 4; i++) so[i] = 0.0;
            log_err(R, 14);
        }
        log_err(R, 15);
    } else {
        for (int i = 0; i < 4; i++) so[i] = si[i];
        log_err(R, 16);
    }
}

// direction_cosine (ARTES.f90:1962-2052)
__device__ void direction_cosine(const DevRun& R, double alpha, double beta, double d0, double d1, double d2,
                                 double& e0, double& e1, double& e2) {
    const double cto = d2 / sqrt(d0 * d0 + d1 * d1 + d2 * d2);
    const double sto = sqrt(1.0 - cto * cto);
    double phi_old = atan2(d1, d0);
    if (phi_old < 0.0) phi_old += TWO_PI;
    double ctn = 0.0, phi_new = 0.0, spn = 0.0;
    const bool upper = (beta >= PI && beta < TWO_PI);
    const bool lower = (beta >= 0.0 && beta < PI);
    if (upper) ctn = cto * alpha + sto * sqrt(1.0 - alpha * alpha) * cos_b(TWO_PI - beta);
    else if (lower) ctn = cto * alpha + sto * sqrt(1.0 - alpha * alpha) * cos_b(beta);
    else log_err(R, 18);
    const double stn = sqrt(1.0 - ctn * ctn);
    double num = (alpha - ctn * cto) / (stn * sto);
    if (num >= 1.0) num = 1.0 - 1.e-10;
    else if (num <= -1.0) num = -1.0 + 1.e-10;
    if (fabs(num) <= 1.0) {
        if (upper) phi_new = phi_old - acos(num);
        else if (lower) phi_new = phi_old + acos(num);
        else log_err(R, 19);
    } else {
        log_err(R, 20);
    }
    if (phi_new < 0.0) phi_new += TWO_PI;
    if (phi_new > TWO_PI) phi_new -= TWO_PI;
    const double cpn = cos_b(phi_new);
    if (phi_new >= 0.0 && phi_new < PI) spn = sqrt(1.0 - cpn * cpn);
    else if (phi_new >= PI && phi_new <= TWO_PI) spn = -sqrt(1.0 - cpn * cpn);
    else log_err(R, 21);
    e0 = stn * cpn;
    e1 = stn * spn;
    e2 = ctn;
}

// linear interpolation of the 16 elements at angle acos(mu) between bin centres
// (ARTES.f90:1448-1530, 4780-4862); P = [180][16] of the cell's matrix
__device__ __forceinline__ void interp_matrix(const double* __restrict__ P, double acos_mu, double sc[16]) {
    const double deg = acos_mu * 180.0 / PI;
    const int ideg = (int)deg;
    int up, lo;
    if (deg - (double)ideg > 0.5) { up = ideg + 2; lo = ideg + 1; }
    else { up = ideg + 1; lo = ideg; }
    if (up == 1) {
#pragma unroll
        for (int i = 0; i < 16; i++) sc[i] = P[i];
    } else if (lo == 180) {
#pragma unroll
        for (int i = 0; i < 16; i++) sc[i] = P[179 * 16 + i];
    } else {
        const double* x0 = P + (lo - 1) * 16;
        const double* x1 = P + (up - 1) * 16;
        const double y0 = (double)lo - 0.5, y1 = (double)up - 0.5;
        const double f = (deg - y0) / (y1 - y0);
#pragma unroll
        for (int i = 0; i < 16; i++) sc[i] = (x1[i] - x0[i]) * f + x0[i];
    }
}

// smallest i in [1,180] with C(i) >= s for a non-decreasing C given by `cdf(i)`
template <typename F>
__device__ __forceinline__ int cdf_search(double s, F cdf) {
    int lo = 1, hi = 180;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (cdf(mid) >= s) hi = mid;
            else lo = mid + 1;
        }
    }
    return lo;
}

// scattering_angle_sampling (ARTES.f90:1534-1661) by binary search on the cumulative tables
__device__ void sample_angles(const DevGrid& G, const DevRun& R, const double* __restrict__ C, Rng& rng,
                              const double st[4], double& alpha, double& beta) {
    // azimuth: C_b(i) = i (p11 I + p14 V) + (p12 Q + p13 U) SC2(i) + (p12 U - p13 Q) SS2(i)
    const double p11 = C[180 * 4 + 0], p12 = C[180 * 4 + 1], p13 = C[180 * 4 + 2], p14 = C[180 * 4 + 3];
    const double u = p11 * st[0] + p14 * st[3];
    const double v = p12 * st[1] + p13 * st[2];
    const double w = p12 * st[2] - p13 * st[1];
    auto cb = [&](int i) { return (double)i * u + v * G.sc2[i] + w * G.ss2[i]; };
    double s = rng.uni() * cb(180);
    int i = cdf_search(s, cb);
    double y0 = cb(i - 1), y1 = cb(i);
    beta = (s - y0) / (y1 - y0) + (double)(i - 1);
    beta = beta * PI / 180.0;
    if (rng.uni() > 0.5) beta = beta + PI;
    if (beta >= TWO_PI) beta = TWO_PI - 1.e-10;
    if (beta <= 0.0) beta = -TWO_PI + 1.e-10;
    double c2b, s2b;
    mueller(beta, c2b, s2b);
    // polar: C_t(i) = I A1(i) + (c2b Q + s2b U) A2(i) + (c2b U - s2b Q) A3(i) + V A4(i)
    const double k0 = st[0], k1 = c2b * st[1] + s2b * st[2], k2 = c2b * st[2] - s2b * st[1], k3 = st[3];
    auto ct = [&](int j) {
        const double* a = C + j * 4;
        return k0 * a[0] + k1 * a[1] + k2 * a[2] + k3 * a[3];
    };
    s = rng.uni() * ct(180);
    i = cdf_search(s, ct);
    y0 = ct(i - 1);
    y1 = ct(i);
    const double adeg = (s - y0) / (y1 - y0) + (double)(i - 1);
    alpha = cos_b(adeg * PI / 180.0);
    if (fabs(alpha) >= 1.0) log_err(R, 56);
    if (alpha >= 1.0) alpha = 1.0 - 1.e-10;
    if (alpha <= -1.0) alpha = -1.0 + 1.e-10;
}

// ------------------------------------------------------------ the kernel ---
enum Mode : int { M_NEW = 0, M_FIRST, M_PROP, M_PEEL, M_EV_FIRST, M_EV_INTERACT, M_EV_PEEL, M_DONE };
enum End : int { E_NONE = -1, E_EXIT = 1, E_ABSORBED = 2, E_DROPPED = 3 };

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

template <bool G3D, bool TRACE>
__global__ __launch_bounds__(BLOCK) void transport_kernel(DevGrid G, DevRun R) {
    const uint64_t nthreads = (uint64_t)gridDim.x * BLOCK;
    uint64_t next = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;   // static interleaved share
    double* __restrict__ det = R.det + (size_t)(blockIdx.x % NCOPY) * R.det_stride;
    const size_t plane = (size_t)R.nx * R.ny;

    // per-lane packet-level moments and per-block counters live in LDS (they are touched
    // only at peel / packet-end events, so they do not need to occupy VGPRs in the hot loop)
    __shared__ double s_cs[4][BLOCK];      // running contribution of the packet to s_pix
    __shared__ double s_pt[4][BLOCK];      // packet total per Stokes
    __shared__ int s_pix[BLOCK];
    __shared__ unsigned long long s_cnt[ARTES_NUM_COUNTERS];
    __shared__ double s_tot2[4];
    const int lane = threadIdx.x;
    if (lane < ARTES_NUM_COUNTERS) s_cnt[lane] = 0ULL;
    if (lane < 4) s_tot2[lane] = 0.0;
#pragma unroll
    for (int k = 0; k < 4; k++) { s_cs[k][lane] = 0.0; s_pt[k][lane] = 0.0; }
    s_pix[lane] = -1;
    __syncthreads();
    uint32_t c_cross = 0;

    // packet state
    Rng rng;
    rng.s0 = rng.s1 = 0;
    uint64_t pid = 0;
    double px = 0, py = 0, pz = 0, dx = 0, dy = 0, dz = 0;
    double st[4] = {0, 0, 0, 0};
    int cr = 0, ct = 0, cp = 0, ft = 0, fi = 0;
    // trace state
    double tx = 0, ty = 0, tz = 0, tau_acc = 0, tau_tgt = 0;
    int tcr = 0, tct = 0, tcp = 0, tft = 0, tfi = 0;
    bool t_exit = false, t_err = false, t_surf = false;
    // trace-record bookkeeping (TRACE builds)
    double rec_peel = 0.0;
    uint32_t rec_scat = 0, rec_cross = 0;
    int endst = E_NONE;
    bool have_pkt = false;
    int mode = M_NEW;

    for (;;) {
        // ================================================================ events
        if (mode == M_EV_FIRST) {   // first optical depth known (ARTES.f90:658-685)
            double tau;
            if (tau_acc < 1.e-6 && !t_surf) {
                mode = M_NEW; endst = E_DROPPED;
            } else {
                const double xi = rng.uni();
                if (tau_acc < 1.e-6) {
                    tau = -log(1.0 - xi);
                } else if (tau_acc < 50.0) {
                    const double e = 1.0 - exp(-tau_acc);
                    tau = -log(1.0 - xi * e);
                    st[0] *= e; st[1] *= e; st[2] *= e; st[3] *= e;
                } else {
                    tau = -log(1.0 - xi);
                }
                tx = px; ty = py; tz = pz;
                tcr = cr; tct = ct; tcp = cp; tft = ft; tfi = fi;
                tau_acc = 0.0; tau_tgt = tau;
                mode = M_PROP;
            }
        }
        if (mode == M_EV_INTERACT) {   // scattering-loop head (ARTES.f90:788-815)
            bool stop = !R.photon_scattering;
            if (!stop) stop = rng.uni() < R.fstop;
            if (!stop) {
                const double alb = G.albedo[cr + G.nr * (ct + G.ntheta * cp)];
                if (alb < 1.0 && alb > 0.0) {
                    const double gamma = alb / (1.0 - R.fstop);
                    st[0] *= gamma; st[1] *= gamma; st[2] *= gamma; st[3] *= gamma;
                }
                if (st[0] <= R.pmin) stop = true;
            }
            if (stop) {
                mode = M_NEW; endst = E_ABSORBED;
            } else {   // start the peel-off trace toward the detector (ARTES.f90:4722-4761)
                atomicAdd(&s_cnt[ARTES_CNT_PEELS], 1ULL);
                tx = px; ty = py; tz = pz;
                tcr = cr; tct = ct; tcp = cp; tft = ft; tfi = fi;
                tau_acc = 0.0;
                mode = M_PEEL;
            }
        }
        // deferral of the peel/scatter event: run it when enough lanes of the wave wait
        // for it, or when no lane is tracing (wave-uniform decision)
        {
            const bool waiting = (mode == M_EV_PEEL);
            const bool tracing = (mode == M_FIRST || mode == M_PROP || mode == M_PEEL);
            const unsigned long long wmask = __ballot(waiting);
            const unsigned long long tmask = __ballot(tracing);
            const bool run_ev = wmask != 0 && (__popcll(wmask) >= R.defer || tmask == 0);
            if (run_ev && waiting) {
                bool drop = t_err;
                if (!drop && t_exit && tau_acc < 50.0) {   // peel contribution (ARTES.f90:4765-4984)
                    const double w = exp(-tau_acc);
                    double mu = dx * R.det0 + dy * R.det1 + dz * R.det2;
                    if (mu >= 1.0) mu = 1.0 - 1.e-10;
                    else if (mu <= -1.0) mu = -1.0 + 1.e-10;
                    const int cell = cr + G.nr * (ct + G.ntheta * cp);
                    const double* __restrict__ P = G.mats + (size_t)G.matid[cell] * MAT_DOUBLES;
                    double sc[16];
                    interp_matrix(P, acos(mu), sc);
                    double phi_old = atan2(dy, dx);
                    if (phi_old < 0.0) phi_old += TWO_PI;
                    if (phi_old > TWO_PI) phi_old -= TWO_PI;
                    double phi_new = atan2(R.det1, R.det0);
                    if (phi_new < 0.0) phi_new += TWO_PI;
                    if (phi_new > TWO_PI) phi_new -= TWO_PI;
                    bool have_out = false;
                    double so[4] = {0, 0, 0, 0};
                    if (fabs(dz) < 1.0) {
                        const double num = (R.det2 - dz * mu) / (sqrt(1.0 - mu * mu) * sqrt(1.0 - dz * dz));
                        double phs = 0.0;
                        if (fabs(num) < 1.0) phs = acos(num);
                        else if (num >= 1.0) phs = 1.e-10;
                        else if (num <= -1.0) phs = PI - 1.e-10;
                        else log_err(R, 44);
                        if (phi_old - phi_new >= 0.0 && phi_old - phi_new < PI) phs = TWO_PI - phs;
                        if (TWO_PI + phi_old - phi_new >= 0.0 && TWO_PI + phi_old - phi_new < PI) phs = TWO_PI - phs;
                        if (phs < 0.0) phs += TWO_PI;
                        if (fabs(mu) < 1.0) {
                            polarization_rotation(R, mu, phs, st, sc, dz, R.det2, so, true);
                            have_out = true;
                        } else {
                            log_err(R, 49);
                            drop = true;
                        }
                    } else {
                        log_err(R, 45);
                    }
                    if (have_out && !drop) {
                        const double x_im = py * R.cdp - px * R.sdp;
                        const double y_im = pz * R.sdt - py * R.cdt * R.sdp - px * R.cdt * R.cdp;
                        const int ix = (int)((double)R.nx * (x_im + R.x_max) / (2.0 * R.x_max));
                        const int iy = (int)((double)R.ny * (y_im + R.y_max) / (2.0 * R.y_max));
                        const double wI = w * so[0];
                        if (wI > 0.0 && wI < 1.e100) {
                            if (ix < 0 || ix >= R.nx || iy < 0 || iy >= R.ny) {
                                log_err(R, 63);
                            } else {
                                const int pix = iy * R.nx + ix;
                                const double v[4] = {w * so[0], -w * so[1], w * so[2], w * so[3]};   // -Q: ARTES.f90:4956
                                const int cur = s_pix[lane];
                                if (pix != cur) {
                                    if (cur >= 0) {
#pragma unroll
                                        for (int k = 0; k < 4; k++) { unsafeAtomicAdd(&det[(12 + k) * plane + cur], s_cs[k][lane] * s_cs[k][lane]); s_cs[k][lane] = 0.0; }
                                    }
                                    s_pix[lane] = pix;
                                }
#pragma unroll
                                for (int k = 0; k < 4; k++) {
                                    unsafeAtomicAdd(&det[k * plane + pix], v[k]);
                                    unsafeAtomicAdd(&det[(4 + k) * plane + pix], v[k] * v[k]);
                                    s_cs[k][lane] += v[k];
                                    s_pt[k][lane] += v[k];
                                }
                                unsafeAtomicAdd(&det[8 * plane + pix], 1.0);
                                atomicAdd(&s_cnt[ARTES_CNT_DETECTED], 1ULL);
                                if constexpr (TRACE) rec_peel += wI;
                            }
                        } else {
                            log_err(R, 53);
                        }
                    }
                }
                if (drop) {
                    mode = M_NEW; endst = E_DROPPED;
                } else {   // scatter_photon + polarization_rotation (ARTES.f90:819-846, 1434-1532)
                    atomicAdd(&s_cnt[ARTES_CNT_SCATTERS], 1ULL);
                    if constexpr (TRACE) rec_scat++;
                    const int cell = cr + G.nr * (ct + G.ntheta * cp);
                    const int m = G.matid[cell];
                    double alpha, beta;
                    sample_angles(G, R, G.cums + (size_t)m * CUM_DOUBLES, rng, st, alpha, beta);
                    double e0, e1, e2;
                    direction_cosine(R, alpha, beta, dx, dy, dz, e0, e1, e2);
                    double sc[16];
                    interp_matrix(G.mats + (size_t)m * MAT_DOUBLES, acos(alpha), sc);
                    if (fabs(alpha) < 1.0) {
                        double sn[4];
                        polarization_rotation(R, alpha, beta, st, sc, dz, e2, sn, false);
                        st[0] = sn[0]; st[1] = sn[1]; st[2] = sn[2]; st[3] = sn[3];
                        dx = e0; dy = e1; dz = e2;
                        const double xi = rng.uni();
                        tx = px; ty = py; tz = pz;
                        tcr = cr; tct = ct; tcp = cp; tft = ft; tfi = fi;
                        tau_acc = 0.0; tau_tgt = -log(1.0 - xi);
                        mode = M_PROP;
                    } else {
                        log_err(R, 50);
                        mode = M_NEW; endst = E_DROPPED;
                    }
                }
            }
        }
        if (mode == M_NEW) {   // close the previous packet, start the next (ARTES.f90:546-597)
            if (have_pkt) {
                atomicAdd(&s_cnt[endst == E_EXIT ? ARTES_CNT_EXITED : (endst == E_ABSORBED ? ARTES_CNT_ABSORBED : ARTES_CNT_DROPPED)], 1ULL);
                const int cur = s_pix[lane];
                if (cur >= 0) {
#pragma unroll
                    for (int k = 0; k < 4; k++) { unsafeAtomicAdd(&det[(12 + k) * plane + cur], s_cs[k][lane] * s_cs[k][lane]); s_cs[k][lane] = 0.0; }
                    s_pix[lane] = -1;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double t = s_pt[k][lane];
                    if (t != 0.0) atomicAdd(&s_tot2[k], t * t);
                    s_pt[k][lane] = 0.0;
                }
                if constexpr (TRACE) {
                    double* rr = R.rec + (size_t)(pid - R.first) * 4;
                    rr[0] = rec_peel; rr[1] = (double)rec_scat; rr[2] = (double)rec_cross; rr[3] = (double)endst;
                    rec_peel = 0.0; rec_scat = 0; rec_cross = 0;
                }
                have_pkt = false;
            }
            if (next < R.n) {
                pid = R.first + next;
                next += nthreads;
                have_pkt = true;
                endst = E_NONE;
                atomicAdd(&s_cnt[ARTES_CNT_PACKETS], 1ULL);
                rng.seed(R.seed, pid);
                // emit_photon, star branch (ARTES.f90:1027-1115)
                const double Rt = G.rtop;
                double r_disk, phi_disk;
                if (R.phase_far) {
                    do { r_disk = sqrt(rng.uni()); } while (!(r_disk > 0.9));
                    phi_disk = TWO_PI * rng.uni();
                } else {
                    r_disk = sqrt(rng.uni());
                    phi_disk = TWO_PI * rng.uni();
                }
                const double d1 = Rt * r_disk * sin_b(phi_disk), d2 = Rt * r_disk * cos_b(phi_disk);
                dx = -1.0; dy = 0.0; dz = 0.0;
                px = sqrt(Rt * Rt - d1 * d1 - d2 * d2); py = d1; pz = d2;
                if (R.stellar_direction) {   // ARTES.f90:1080-1111
                    double c = cos_b(-(HALF_PI - R.theta_star)), s = sin_b(-(HALF_PI - R.theta_star));
                    const double x1 = c * px + s * pz, y1 = py, z1 = -s * px + c * pz;
                    c = cos_b(R.phi_star); s = sin_b(R.phi_star);
                    px = c * x1 - s * y1; py = s * x1 + c * y1; pz = z1;
                    double td = PI - R.theta_star, pd = PI + R.phi_star;
                    if (td < 0.0) td += TWO_PI;
                    if (td > TWO_PI) td -= TWO_PI;
                    if (pd < 0.0) pd += TWO_PI;
                    if (pd > TWO_PI) pd -= TWO_PI;
                    dx = sin_b(td) * cos_b(pd); dy = sin_b(td) * sin_b(pd); dz = cos_b(td);
                }
                // initial_cell (ARTES.f90:2605-2669)
                cr = G.nr - 1; ct = 0; cp = 0;
                if constexpr (G3D) {
                    const double r = sqrt(px * px + py * py + pz * pz);
                    const double th = acos(pz / r);
                    double ph = atan2(py, px);
                    if (ph < 0.0) ph += TWO_PI;
                    for (int j = 0; j < G.ntheta; j++)
                        if (th > G.thetaf[j] && th < G.thetaf[j + 1]) { ct = j; break; }
                    for (int j = 0; j < G.nphi; j++) {
                        const double hi = (j < G.nphi - 1) ? G.phif[j + 1] : TWO_PI;
                        if (ph > G.phif[j] && ph < hi) { cp = j; break; }
                    }
                }
                ft = 1; fi = G.nr;
                st[0] = 1.0; st[1] = 0.0; st[2] = 0.0; st[3] = 0.0;
                tx = px; ty = py; tz = pz;
                tcr = cr; tct = ct; tcp = cp; tft = ft; tfi = fi;
                tau_acc = 0.0;
                mode = M_FIRST;
            } else {
                mode = M_DONE;
            }
        }
        if (__all(mode == M_DONE)) break;

        // ============================================================ trace step
        if (mode == M_FIRST || mode == M_PROP || mode == M_PEEL) {
            const bool peel = (mode == M_PEEL);   // trace direction: detector for peel-off, else the packet's
            const double tdx = peel ? R.det0 : dx, tdy = peel ? R.det1 : dy, tdz = peel ? R.det2 : dz;
            Step o;
            cell_face<G3D>(G, R, tx, ty, tz, tdx, tdy, tdz, tft, tfi, tcr, tct, tcp, o);
            c_cross++;
            if constexpr (TRACE) rec_cross++;
            const double k = G.kappa[tcr + G.nr * (tct + G.ntheta * tcp)];
            const double tau_cell = o.d * k;
            const bool surf = (o.nft == 1 && o.nfi == G.cell_depth);
            if (mode == M_PROP) {   // ARTES.f90:691-778 / 850-941
                if (o.err) {
                    log_err(R, 3);
                    mode = M_NEW; endst = E_DROPPED;
                } else if (tau_acc + tau_cell > tau_tgt) {
                    const double s = (tau_tgt - tau_acc) / k;
                    px = tx + s * tdx; py = ty + s * tdy; pz = tz + s * tdz;
                    cr = tcr; ct = tct; cp = tcp; ft = 0; fi = 0;
                    mode = M_EV_INTERACT;
                } else {
                    tx += o.d * tdx; ty += o.d * tdy; tz += o.d * tdz;
                    tft = o.nft; tfi = o.nfi; tcr = o.ncr; tct = o.nct; tcp = o.ncp;
                    if (o.exit) {
                        mode = M_NEW; endst = E_EXIT;
                    } else if (surf) {
                        if (rng.uni() > R.surface_albedo) { mode = M_NEW; endst = E_ABSORBED; }
                        else { log_err(R, 62); mode = M_NEW; endst = E_DROPPED; }   // Lambertian: not yet supported
                    } else {
                        tau_acc += tau_cell;
                    }
                }
            } else {   // first-tau trace (ARTES.f90:633-656) or peel trace (4739-4761)
                tau_acc += tau_cell;
                tx += o.d * tdx; ty += o.d * tdy; tz += o.d * tdz;
                if (o.err) log_err(R, mode == M_FIRST ? 2 : 43);
                if (o.exit || o.err || surf) {
                    t_exit = o.exit; t_err = o.err; t_surf = surf;
                    mode = (mode == M_FIRST) ? M_EV_FIRST : M_EV_PEEL;
                    if (mode == M_EV_FIRST) t_err = false;   // the reference does not drop on a first-trace error
                } else {
                    tft = o.nft; tfi = o.nfi; tcr = o.ncr; tct = o.nct; tcp = o.ncp;
                }
            }
        }
    }

    // ============================================================= flush
    const unsigned long long w_cross = wave_sum_u64(c_cross);
    if ((lane & 63) == 0) atomicAdd(&s_cnt[ARTES_CNT_CROSSINGS], w_cross);
    __syncthreads();
    if (lane < ARTES_NUM_COUNTERS) atomicAdd(&R.cnt[lane], s_cnt[lane]);
    if (lane < 4) unsafeAtomicAdd(&R.tot2[lane], s_tot2[lane]);
}

// sum the NCOPY privatised detectors into `out` ([4][4][ny][nx], accumulated) and
// replicate the peel count into the four Stokes slots of plane 2 (ARTES.f90:4969-4972)
__global__ void reduce_detector(const double* __restrict__ copies, size_t stride, size_t plane, double* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= stride) return;
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < NCOPY; c++) s += copies[(size_t)c * stride + i];
    const size_t slot = i / plane;           // 0..15 = moment*4 + stokes
    if (slot == 8) {
        const size_t pix = i - 8 * plane;
        out[i] += s;
        out[9 * plane + pix] += s;
        out[10 * plane + pix] += s;
        out[11 * plane + pix] += s;
    } else if (slot == 9 || slot == 10 || slot == 11) {
        // filled from slot 8
    } else {
        out[i] += s;
    }
}

}  // namespace artes

// ================================================================= C ABI ===
using namespace artes;

struct artes_grid {
    int device = 0;
    HostTables T;
    double *d_rf2 = nullptr, *d_thetaf = nullptr, *d_tan2 = nullptr, *d_phif = nullptr, *d_phis = nullptr,
           *d_phic = nullptr, *d_kappa = nullptr, *d_albedo = nullptr, *d_mats = nullptr, *d_cums = nullptr,
           *d_sc2 = nullptr, *d_ss2 = nullptr;
    int *d_tplane = nullptr, *d_matid = nullptr;
    double* d_copies = nullptr;
    size_t copies_cap = 0;
    double* d_out = nullptr;          // scratch outputs for the host-pointer variant
    size_t out_cap = 0;
    double* d_tot = nullptr;
    unsigned long long* d_cnt = nullptr;
    unsigned long long* d_err = nullptr;
    double* d_rec = nullptr;
    size_t rec_cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    int max_blocks = 0;
};

static thread_local std::string g_last_error;

static int32_t fail(int32_t code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess) return fail(-5, std::string(#expr ": ") + hipGetErrorString(_e)); \
    } while (0)

template <typename T>
static hipError_t upload(T** dst, const std::vector<T>& src) {
    hipError_t e = hipMalloc((void**)dst, std::max<size_t>(src.size(), 1) * sizeof(T));
    if (e != hipSuccess) return e;
    if (!src.empty()) e = hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
    return e;
}

extern "C" {

int32_t artes_abi_version(void) { return ARTES_ABI_VERSION; }

const char* artes_build_info(void) {
    return "artes_amd transport engine: gfx950 HIP, FP64, persistent state-machine kernel, NCOPY=8";
}

const char* artes_last_error(void) { return g_last_error.c_str(); }

int32_t artes_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return -5;
    return n;
}

void artes_grid_destroy(artes_grid* g) {
    if (!g) return;
    hipSetDevice(g->device);
    void* ptrs[] = {g->d_rf2, g->d_thetaf, g->d_tan2, g->d_phif, g->d_phis, g->d_phic, g->d_kappa, g->d_albedo,
                    g->d_mats, g->d_cums, g->d_sc2, g->d_ss2, g->d_tplane, g->d_matid, g->d_copies, g->d_out,
                    g->d_tot, g->d_cnt, g->d_err, g->d_rec};
    for (void* p : ptrs)
        if (p) hipFree(p);
    if (g->ev0) hipEventDestroy(g->ev0);
    if (g->ev1) hipEventDestroy(g->ev1);
    delete g;
}

int32_t artes_grid_create(const artes_grid_desc* desc, int32_t device, artes_grid** out) {
    if (!desc || !out) return fail(-22, "null argument");
    *out = nullptr;
    std::unique_ptr<artes_grid> g(new artes_grid());
    g->device = device;
    try {
        g->T = build_tables(*desc);
    } catch (const std::exception& e) {
        return fail(-22, e.what());
    }
    HIP_TRY(hipSetDevice(device));
    const HostTables& T = g->T;
    HIP_TRY(upload(&g->d_rf2, T.rf2));
    HIP_TRY(upload(&g->d_thetaf, T.thetaf));
    HIP_TRY(upload(&g->d_tan2, T.tan2));
    HIP_TRY(upload(&g->d_tplane, T.tplane));
    HIP_TRY(upload(&g->d_phif, T.phif));
    HIP_TRY(upload(&g->d_phis, T.phis));
    HIP_TRY(upload(&g->d_phic, T.phic));
    HIP_TRY(upload(&g->d_kappa, T.kappa));
    HIP_TRY(upload(&g->d_albedo, T.albedo));
    HIP_TRY(upload(&g->d_matid, T.matid));
    HIP_TRY(upload(&g->d_mats, T.mats));
    HIP_TRY(upload(&g->d_cums, T.cums));
    HIP_TRY(upload(&g->d_sc2, T.sc2));
    HIP_TRY(upload(&g->d_ss2, T.ss2));
    HIP_TRY(hipMalloc((void**)&g->d_tot, 4 * sizeof(double)));
    HIP_TRY(hipMalloc((void**)&g->d_cnt, ARTES_NUM_COUNTERS * sizeof(unsigned long long)));
    HIP_TRY(hipMalloc((void**)&g->d_err, ARTES_NUM_ERR * sizeof(unsigned long long)));
    HIP_TRY(hipEventCreate(&g->ev0));
    HIP_TRY(hipEventCreate(&g->ev1));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    int per_cu = 0;
    const bool g3d = (T.ntheta > 1 || T.nphi > 1);
    if (g3d) HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, transport_kernel<true, false>, BLOCK, 0));
    else HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, transport_kernel<false, false>, BLOCK, 0));
    g->max_blocks = std::max(1, per_cu) * prop.multiProcessorCount;
    HIP_TRY(hipDeviceSynchronize());
    *out = g.release();
    return 0;
}

int32_t artes_grid_cell_depth(const artes_grid* g, int32_t wl) {
    if (!g || wl < 0 || wl >= g->T.nwav) return -22;
    return g->T.cell_depth[wl];
}

int32_t artes_grid_num_matrices(const artes_grid* g) { return g ? g->T.nmat : -22; }

static int32_t launch(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                      double* det_out, double* tot_out, unsigned long long* cnt_out, unsigned long long* err_out,
                      double* rec, hipStream_t stream) {
    const HostTables& T = g->T;
    if (!p) return fail(-22, "null params");
    if (p->photon_source != 1) return fail(-38, "photon:source=planet is not implemented in the GPU engine yet");
    if (p->wl_index < 0 || p->wl_index >= T.nwav) return fail(-22, "wl_index out of range");
    if (p->nx < 1 || p->ny < 1 || (size_t)p->nx * p->ny > (1u << 26)) return fail(-22, "bad detector size");
    if (p->surface_albedo > 0.0) return fail(-38, "planet:surface_albedo > 0 (Lambertian surface) is not implemented yet");
    HIP_TRY(hipSetDevice(g->device));
    const size_t plane = (size_t)p->nx * p->ny;
    const size_t stride = 16 * plane;
    if (g->copies_cap < stride * NCOPY) {
        if (g->d_copies) hipFree(g->d_copies);
        g->d_copies = nullptr;
        HIP_TRY(hipMalloc((void**)&g->d_copies, stride * NCOPY * sizeof(double)));
        g->copies_cap = stride * NCOPY;
    }
    HIP_TRY(hipMemsetAsync(g->d_copies, 0, stride * NCOPY * sizeof(double), stream));

    DevGrid G;
    G.nr = T.nr; G.ntheta = T.ntheta; G.nphi = T.nphi; G.ncell = T.ncell;
    G.cell_depth = p->cell_depth >= 0 ? p->cell_depth : T.cell_depth[p->wl_index];
    G.ax2 = 1.0 / (T.oblate_x * T.oblate_x); G.by2 = 1.0 / (T.oblate_y * T.oblate_y); G.cz2 = 1.0 / (T.oblate_z * T.oblate_z);
    G.a = 1.0 / T.oblate_x; G.b = 1.0 / T.oblate_y;
    G.rtop = T.rfront[T.nr];
    G.rf2 = g->d_rf2; G.thetaf = g->d_thetaf; G.tan2 = g->d_tan2; G.tplane = g->d_tplane;
    G.phif = g->d_phif; G.phis = g->d_phis; G.phic = g->d_phic;
    G.kappa = g->d_kappa + (size_t)p->wl_index * T.ncell;
    G.albedo = g->d_albedo + (size_t)p->wl_index * T.ncell;
    G.matid = g->d_matid + (size_t)p->wl_index * T.ncell;
    G.mats = g->d_mats; G.cums = g->d_cums; G.sc2 = g->d_sc2; G.ss2 = g->d_ss2;

    DevRun R;
    R.first = first; R.n = n; R.seed = seed;
    R.nx = p->nx; R.ny = p->ny; R.photon_scattering = p->photon_scattering; R.phase_far = p->phase_far;
    R.stellar_direction = p->stellar_direction;
    const char* env = getenv("ARTES_DEFER");
    R.defer = env ? atoi(env) : 16;
    R.det0 = sin(p->det_theta) * cos(p->det_phi);   // spherical_cartesian (ARTES.f90:495)
    R.det1 = sin(p->det_theta) * sin(p->det_phi);
    R.det2 = cos(p->det_theta);
    R.sdt = sin(p->det_theta); R.cdt = cos(p->det_theta); R.sdp = sin(p->det_phi); R.cdp = cos(p->det_phi);
    R.x_max = p->x_max; R.y_max = p->y_max; R.fstop = p->fstop; R.pmin = p->photon_minimum;
    R.surface_albedo = p->surface_albedo; R.theta_star = p->theta_star; R.phi_star = p->phi_star;
    R.det = g->d_copies; R.det_stride = stride;
    R.tot2 = tot_out; R.cnt = cnt_out; R.err = err_out; R.rec = rec;

    const bool g3d = (T.ntheta > 1 || T.nphi > 1);
    uint64_t want = (n + BLOCK - 1) / BLOCK;
    int blocks = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)g->max_blocks));
    HIP_TRY(hipEventRecord(g->ev0, stream));
    if (n > 0) {
        if (rec) {
            if (g3d) hipLaunchKernelGGL((transport_kernel<true, true>), dim3(blocks), dim3(BLOCK), 0, stream, G, R);
            else hipLaunchKernelGGL((transport_kernel<false, true>), dim3(blocks), dim3(BLOCK), 0, stream, G, R);
        } else {
            if (g3d) hipLaunchKernelGGL((transport_kernel<true, false>), dim3(blocks), dim3(BLOCK), 0, stream, G, R);
            else hipLaunchKernelGGL((transport_kernel<false, false>), dim3(blocks), dim3(BLOCK), 0, stream, G, R);
        }
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipEventRecord(g->ev1, stream));
    g->timed = true;
    const int rb = (int)((stride + 255) / 256);
    hipLaunchKernelGGL(reduce_detector, dim3(rb), dim3(256), 0, stream, (const double*)g->d_copies, stride, plane, det_out);
    HIP_TRY(hipGetLastError());
    return 0;
}

int32_t artes_run_device(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                         double* det_dev, double* tot_dev, uint64_t* cnt_dev, uint64_t* err_dev, void* stream) {
    if (!g || !det_dev) return fail(-22, "null argument");
    HIP_TRY(hipSetDevice(g->device));
    hipStream_t s = (hipStream_t)stream;
    if (!tot_dev) { HIP_TRY(hipMemsetAsync(g->d_tot, 0, 4 * sizeof(double), s)); }
    if (!cnt_dev) { HIP_TRY(hipMemsetAsync(g->d_cnt, 0, ARTES_NUM_COUNTERS * 8, s)); }
    if (!err_dev) { HIP_TRY(hipMemsetAsync(g->d_err, 0, ARTES_NUM_ERR * 8, s)); }
    return launch(g, p, first, n, seed, det_dev, tot_dev ? tot_dev : g->d_tot,
                  cnt_dev ? (unsigned long long*)cnt_dev : g->d_cnt, err_dev ? (unsigned long long*)err_dev : g->d_err,
                  nullptr, s);
}

static int32_t run_host(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                        double* det, double* totals, uint64_t* counters, uint64_t* err, double* records) {
    if (!g || !p) return fail(-22, "null argument");
    HIP_TRY(hipSetDevice(g->device));
    const size_t stride = (size_t)16 * p->nx * p->ny;
    if (g->out_cap < stride) {
        if (g->d_out) hipFree(g->d_out);
        g->d_out = nullptr;
        HIP_TRY(hipMalloc((void**)&g->d_out, stride * sizeof(double)));
        g->out_cap = stride;
    }
    if (records) {
        if (g->rec_cap < n * 4) {
            if (g->d_rec) hipFree(g->d_rec);
            g->d_rec = nullptr;
            HIP_TRY(hipMalloc((void**)&g->d_rec, std::max<uint64_t>(n, 1) * 4 * sizeof(double)));
            g->rec_cap = n * 4;
        }
        HIP_TRY(hipMemset(g->d_rec, 0, std::max<uint64_t>(n, 1) * 4 * sizeof(double)));
    }
    HIP_TRY(hipMemset(g->d_out, 0, stride * sizeof(double)));
    HIP_TRY(hipMemset(g->d_tot, 0, 4 * sizeof(double)));
    HIP_TRY(hipMemset(g->d_cnt, 0, ARTES_NUM_COUNTERS * 8));
    HIP_TRY(hipMemset(g->d_err, 0, ARTES_NUM_ERR * 8));
    int32_t rc = launch(g, p, first, n, seed, g->d_out, g->d_tot, g->d_cnt, g->d_err, records ? g->d_rec : nullptr, 0);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    std::vector<double> hd(stride);
    HIP_TRY(hipMemcpy(hd.data(), g->d_out, stride * sizeof(double), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < stride; i++) det[i] += hd[i];
    if (totals) {
        double t2[4];
        HIP_TRY(hipMemcpy(t2, g->d_tot, sizeof(t2), hipMemcpyDeviceToHost));
        const size_t plane = (size_t)p->nx * p->ny;
        for (int k = 0; k < 4; k++) {
            double s = 0.0;
            for (size_t i = 0; i < plane; i++) s += hd[k * plane + i];
            totals[k] += s;
            totals[4 + k] += t2[k];
        }
    }
    if (counters) {
        unsigned long long c[ARTES_NUM_COUNTERS];
        HIP_TRY(hipMemcpy(c, g->d_cnt, sizeof(c), hipMemcpyDeviceToHost));
        for (int i = 0; i < ARTES_NUM_COUNTERS; i++) counters[i] += c[i];
    }
    if (err) {
        unsigned long long e[ARTES_NUM_ERR];
        HIP_TRY(hipMemcpy(e, g->d_err, sizeof(e), hipMemcpyDeviceToHost));
        for (int i = 0; i < ARTES_NUM_ERR; i++) err[i] += e[i];
    }
    if (records) HIP_TRY(hipMemcpy(records, g->d_rec, n * 4 * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

int32_t artes_run(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                  double* det, double* totals, uint64_t* counters, uint64_t* err) {
    if (!det) return fail(-22, "null detector");
    return run_host(g, p, first, n, seed, det, totals, counters, err, nullptr);
}

int32_t artes_run_trace(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                        double* records) {
    if (!records) return fail(-22, "null records");
    if (n > (1ull << 24)) return fail(-22, "trace runs are limited to 2^24 packets");
    std::vector<double> det((size_t)16 * p->nx * p->ny, 0.0);
    return run_host(g, p, first, n, seed, det.data(), nullptr, nullptr, nullptr, records);
}

double artes_last_kernel_ms(artes_grid* g) {
    if (!g || !g->timed) return -1.0;
    float ms = -1.0f;
    if (hipEventElapsedTime(&ms, g->ev0, g->ev1) != hipSuccess) return -1.0;
    return (double)ms;
}

}  // extern "C"
