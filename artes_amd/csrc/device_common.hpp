// device_common.hpp -- device-side building blocks shared by the transport kernels:
// grid/run descriptors, the per-packet RNG, bounded sin/cos, the cell-face geometry
// (ARTES.f90:2671-3470) and the scattering physics (ARTES.f90:1434-2052).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "tables.hpp"

namespace artes {

// privatised detector copies: up to NCOPY_MAX, copy = block index mod R.ncopy (a multiple of
// 8, so one copy serves the blocks of one XCD); det_copies() picks how many (transport.hip)
constexpr int NCOPY_MAX = 64;
constexpr int BLOCK = 256;
constexpr double PI = 3.14159265358979323846;
constexpr double HALF_PI = PI / 2.0;
constexpr double TWO_PI = 2.0 * PI;

// -------------------------------------------------------------- device data ---
struct DevGrid {
    int nr, ntheta, nphi, ncell, nmat;
    int msym;                            // mats holds the block-diagonal symmetric form (interp_matrix)
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
    const double* __restrict__ ka;       // [ncell][2]: extinction, albedo weight (k_trace: one 16-byte load per step)
    const int* __restrict__ matid;       // [ncell]
    const double* __restrict__ mats;     // [nmat][180][16], or with msym [nmat][180][4] = (P11, P12, P33, P34)
    const double* __restrict__ cums;     // [nmat][181][4]
    const double* __restrict__ sc2;      // [181]
    const double* __restrict__ ss2;      // [181]
    // thermal source and surface (photon:source=planet, planet:surface_albedo)
    const double* __restrict__ rfr;      // rfront [nr+1]
    const double* __restrict__ tcos;     // cos(theta_f) [ntheta+1]
    const double* __restrict__ th_cdf;   // emissivity CDF [(nr-cell_depth)*ntheta*nphi], order (i, j, k)
    const double* __restrict__ th_weight;   // cell_weight [ncell]
    int th_ncdf, th_cd0;                 // CDF length; radial index of its first entry
    double th_total;
    double ox, oy, oz;                   // oblate_x, oblate_y, oblate_z (ARTES.f90:469-471)
    double* ttab;                        // k_trace's face tables in global memory (GTAB kernels: tables beyond 64 KiB), or null
};

struct DevRun {
    uint64_t first, n, seed;
    int nx, ny, photon_scattering, phase_far, stellar_direction, defer, refill, static_q64, batch, batch_min, hbatch;
    int late_append;                // k_trace: list appends of ended chains at the wave's next refill (kernel_trace.hpp)
    int gbatch;                     // k_trace (trace-relative): theta / phi evaluations run once this many lanes wait
    int dgrab;                      // k_trace: the least list entries a dynamic (atomic) grab asks for
    int photon_source, photon_emission;
    int moments;                    // accumulate packet-level moments (slot line 1, planes 12-15, tot2[0..3])
    int emit_first;                 // trace-list order (kernel_event.hpp, Lists)
    int backward;                   // k_trace: backward propagation after the forced interaction
    double photon_bias;
    double det0, det1, det2, sdt, cdt, sdp, cdp;
    double det_phi;                 // atan2(det1, det0) in [0, 2 pi] (peel_photon, ARTES.f90:4868-4870)
    double cdphi, sdphi;            // its cosine and sine
    double x_max, y_max, fstop, pmin, surface_albedo, theta_star, phi_star;
    double* __restrict__ det;       // [ncopy][4][4][ny][nx], copies det_stride doubles apart
    size_t det_stride;              // doubles per copy (16 ny nx rounded up to 256 bytes)
    int ncopy;                      // detector copies
    unsigned long long* __restrict__ fix;   // det_ordered: [nfix][10][ny][nx] 128-bit fixed-point planes 0-9 (lo, hi), or null
    size_t fix_stride;              // u64 per fixed-point copy (20 ny nx)
    int nfix;                       // fixed-point copies (copy = block index mod nfix)
    double* __restrict__ tot2;      // [CNT_COPIES][CNT_STRIDE] partials (tot_add) of: packet-level sum T^2 per Stokes, flux_emitted, flux_exit
    unsigned long long* __restrict__ cnt;   // [CNT_COPIES][CNT_STRIDE] partial counters (cnt_add), summed per call
    unsigned long long* __restrict__ err;   // [ARTES_NUM_ERR]
    double* __restrict__ rec;       // [n][ARTES_TRACE_FIELDS] (TRACE builds)
    double* __restrict__ flow_g;    // [ncell][3] flow_global accumulators, or null
    double* __restrict__ flow_t;    // [ncell][4] flow_latitudinal accumulators, or null
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

// The event counters are added once per wave at the end of every launch -- thousands of
// same-address atomics per launch, which the memory side serialises -- so each block adds
// into one of CNT_COPIES copies of them, 256 bytes apart (copy = block index mod 64: eight
// per XCD), and the host's launch sums the copies into the caller's counters at the end
// of the call (sum_counters, transport.hip).
constexpr int CNT_COPIES = 64, CNT_STRIDE = 32;
__device__ __forceinline__ void cnt_add(const DevRun& R, int k, unsigned long long v) {
    atomicAdd(&R.cnt[(blockIdx.x % CNT_COPIES) * CNT_STRIDE + k], v);
}
// the same for the six per-call float totals (packet moments T^2, thermal fluxes)
__device__ __forceinline__ void tot_add(const DevRun& R, int k, double v) {
    unsafeAtomicAdd(&R.tot2[(blockIdx.x % CNT_COPIES) * CNT_STRIDE + k], v);
}

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
// roots of a s^2 + b s + c = 0 in the cancellation-free form; 0 where a root does not
// exist (negative discriminant, degenerate a or q).  Straight-line code: every lane of a
// wave evaluates it the same way, the conditions only select.
__device__ __forceinline__ void quad_roots(double a, double b, double c, double& s0, double& s1) {
    const double disc = b * b - 4.0 * a * c;
    const bool ok = disc >= 0.0;
    const double q = -0.5 * (b + copysign(sqrt(ok ? disc : 0.0), b));
    const double r0 = q / a, r1 = c / q;
    s0 = (ok && fabs(a) > 1.e-100) ? r0 : 0.0;
    s1 = (ok && fabs(q) > 1.e-100) ? r1 : 0.0;
}
// root selection block of cell_face (e.g. ARTES.f90:2897-2907): the smaller root above
// `tol`, 0 if none, if both are equal or if the choice is >= 1e100.  Written as selects:
// the nested ifs of the reference compile to exec-mask branches on a wave.
__device__ __forceinline__ double pick_root(double s0, double s1, double tol) {
    const bool p0 = s0 > tol, p1 = s1 > tol;
    const double both = (s0 < s1) ? s0 : ((s1 < s0) ? s1 : 0.0);
    double r = (p0 & p1) ? both : 0.0;
    r = (p0 & !p1) ? s0 : r;
    r = (!p0 & p1) ? s1 : r;
    return (r < 1.e100) ? r : 0.0;
}

// theta cone x^2+y^2 = z^2 tan^2(theta_f) with the nappe filter (ARTES.f90:3026-3064)
template <bool OBL>
__device__ __forceinline__ double cone_distance(const DevGrid& G, int f, double x, double y, double z,
                                                double n0, double n1, double n2, double tol) {
    // spheroid axis factors; exactly 1 for a spherical planet (OBL = false), where the
    // products they appear in are exact and fold away
    const double ax2 = OBL ? G.ax2 : 1.0, by2 = OBL ? G.by2 : 1.0, cz2 = OBL ? G.cz2 : 1.0;
    const double t2 = G.tan2[f];
    const double qa = ax2 * n0 * n0 + by2 * n1 * n1 - cz2 * n2 * n2 * t2;
    const double qb = 2.0 * (ax2 * x * n0 + by2 * y * n1 - cz2 * z * n2 * t2);
    const double qc = ax2 * x * x + by2 * y * y - cz2 * z * z * t2;
    double s0, s1;
    quad_roots(qa, qb, qc, s0, s1);
    const double th = G.thetaf[f];
    const double z0 = z + s0 * n2, z1 = z + s1 * n2;
    if (s0 > 1.e-15 && ((z0 > 0.0 && th > HALF_PI) || (z0 < 0.0 && th < HALF_PI))) s0 = 0.0;
    if (s1 > 1.e-15 && ((z1 > 0.0 && th > HALF_PI) || (z1 < 0.0 && th < HALF_PI))) s1 = 0.0;
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
template <bool G3D, bool OBL = true>
__device__ __forceinline__ void cell_face(const DevGrid& G, const DevRun& R, double x, double y, double z,
                                          double n0, double n1, double n2, int ft, int fi, int cr, int ct, int cp,
                                          Step& o) {
    const double ax2 = OBL ? G.ax2 : 1.0, by2 = OBL ? G.by2 : 1.0, cz2 = OBL ? G.cz2 : 1.0;
    const double ga = OBL ? G.a : 1.0, gb = OBL ? G.b : 1.0;
    // Every candidate face is evaluated unconditionally and the reference's case split
    // (same face / cone / 90-degree plane / no face) only selects among the results:
    // lanes of a wave sit on different face kinds, and branching on them would run the
    // divergent variants one after another.
    const double qa = ax2 * n0 * n0 + by2 * n1 * n1 + cz2 * n2 * n2;
    const double qb = 2.0 * (ax2 * x * n0 + by2 * y * n1 + cz2 * z * n2);
    const double S = ax2 * x * x + by2 * y * y + cz2 * z * z;
    double s0, s1;
    quad_roots(qa, qb, S - G.rf2[cr], s0, s1);        // inner sphere r_cell
    const double d_rin = (ft == 1 && fi == cr) ? 0.0 : pick_root(s0, s1, 1.e-15);
    quad_roots(qa, qb, S - G.rf2[cr + 1], s0, s1);    // outer sphere r_cell+1 (same face: 1e-3)
    const double d_rout = pick_root(s0, s1, (ft == 1 && fi == cr + 1) ? 1.e-3 : 1.e-15);
    double d_tin = 0.0, d_tout = 0.0, d_pin = 0.0, d_pout = 0.0;
    int pout = 0;
    if constexpr (G3D) {
        const bool on_t = (ft == 2);
        const double zp = -z / n2;                     // the 90-degree face is the plane z = 0
        {                                              // inner theta face (index ct)
            const bool same = on_t && fi == ct;
            const double dc = cone_distance<OBL>(G, ct, x, y, z, n0, n1, n2, same ? 1.e-3 : 1.e-15);
            double d;
            if (G.tplane[ct] == 1) d = (!same || G.thetaf[ct] > HALF_PI) ? dc : 0.0;
            else d = (!same && zp > 0.0 && n2 > 1.e-15) ? zp : 0.0;
            d_tin = (ct != 0) ? d : 0.0;
        }
        {                                              // outer theta face (index ct+1)
            const bool same = on_t && fi == ct + 1;
            const double dc = cone_distance<OBL>(G, ct + 1, x, y, z, n0, n1, n2, same ? 1.e-3 : 1.e-15);
            double d;
            if (G.tplane[ct + 1] == 1) d = (!same || G.thetaf[ct + 1] < HALF_PI) ? dc : 0.0;
            else d = (!same && zp > 0.0 && n2 < -1.e-15) ? zp : 0.0;
            d_tout = (ct + 1 != G.ntheta) ? d : 0.0;
        }
        if (G.nphi > 1) {                              // phi half-planes (ARTES.f90:3292-3350)
            pout = (cp + 1 == G.nphi) ? 0 : cp + 1;
            const bool on_p = (ft == 3);
            const double den0 = gb * n1 * G.phic[cp] - ga * n0 * G.phis[cp];
            const double num0 = ga * x * G.phis[cp] - gb * y * G.phic[cp];
            const double den1 = gb * n1 * G.phic[pout] - ga * n0 * G.phis[pout];
            const double num1 = ga * x * G.phis[pout] - gb * y * G.phic[pout];
            const double q0 = num0 / den0, q1 = num1 / den1;
            const double sp0 = (!(on_p && fi == cp) && fabs(den0) > 0.0) ? q0 : 0.0;
            d_pin = (sp0 > 1.e-15 && sp0 < 1.e100) ? sp0 : 0.0;
            const bool ok1 = !(on_p && fi == pout) && fabs(den1) > 0.0;
            d_pout = (ok1 && q1 > 1.e-15 && sp0 < 1.e100) ? q1 : 0.0;   // sic: sp0 (ARTES.f90:3318, 3346)
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
// sqrt to ~1 ulp for the scattering geometry: the v_rsq_f64 seed, one Newton step on
// (sqrt, 1/(2 sqrt)) and one residual correction -- 9 instructions against ~25 for the
// correctly rounded lowering; +0 for +0, NaN below 0 (as sqrt)
__device__ __forceinline__ double dsqrt(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
    const double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    const double d = fma(-g, g, x);
    g = fma(d, h, g);
    return x > 0.0 ? g : (x == 0.0 ? x : __builtin_nan(""));
}

// the correctly rounded square root (as the reference's sqrt): where a rounding decides a branch
// (direction_cosine_cs, peel_rotation)
__device__ __forceinline__ double ref_sqrt(double x) { return __builtin_sqrt(x); }

// mueller_matrix_filler (ARTES.f90:1934-1960): returns c2p, s2p
__device__ __forceinline__ void mueller(double psi, double& c2p, double& s2p) {
    c2p = cos_b(2.0 * psi);
    s2p = dsqrt(1.0 - c2p * c2p);
    if ((psi > HALF_PI && psi < PI) || (psi > 1.5 * PI && psi < TWO_PI) || (psi > -HALF_PI && psi < 0.0) ||
        (psi > -TWO_PI && psi < -1.5 * PI))
        s2p = -s2p;
}

// polarization_rotation (ARTES.f90:1663-1932); sc is scatter(4,4) row-major.  The first
// rotation is mueller(beta) = (c2b, s2b) (ARTES.f90:1934-1960), and beta's half-turn decides
// the rotation back: rot_lo = beta in [0, pi), rot_hi = beta in [pi, 2 pi) (neither: none).
// The angle back, beta2 = acos(num) (1730-1751), is used only through mueller(+-beta2), i.e.
// cos(2 beta2) = 2 num^2 - 1 and the sine's sign by beta2's quadrant, which is num's sign
// (beta2 in (pi/2, pi) <=> num in (-1, 0)): no acos and no cosine of the angle.  (The
// reference rounds through the angle; the two agree to ~1e-16 absolute, except that the
// quadrant test sees num's sign where the rounded acos(num) may land on pi/2 for
// |num| < 1e-16.)
__device__ void polarization_rotation_cs(const DevRun& R, double alpha, double c2b, double s2b, bool rot_lo, bool rot_hi,
                                         const double si[4], const double sc[16], double d2, double dn2, double so[4],
                                         bool peeling) {
    if (fabs(alpha) < 1.0 && fabs(dn2) < 1.0) {
        double x2 = 1.0;   // cos(beta2); beta2 = 0 unless set (ARTES.f90:1730-1751)
        const double num = (d2 - dn2 * alpha) / (dsqrt(1.0 - alpha * alpha) * dsqrt(1.0 - dn2 * dn2));
        if (fabs(num) <= 1.0) x2 = num;
        else if (num > 1.0 && num < 1.00001) x2 = 1.0;
        else if (num < -1.0 && num > -1.00001) x2 = -1.0;   // beta2 = pi
        else log_err(R, 11);
        double c = c2b, s = s2b;
        double r0 = si[0], r1 = c * si[1] + s * si[2], r2 = -s * si[1] + c * si[2], r3 = si[3];
        const double pr = dsqrt(r1 * r1 + r2 * r2 + r3 * r3);
        double norm = (pr > 0.0) ? dsqrt(si[1] * si[1] + si[2] * si[2] + si[3] * si[3]) / pr : 1.0;
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
        // mueller(beta2) or mueller(-beta2) (ARTES.f90:1905-1910): cos(2 beta2) either way; the
        // sine negative on beta2 in (pi/2, pi) for +beta2 (num in (-1, 0)), on (0, pi/2) for
        // -beta2 (num in (0, 1))
        if (rot_lo || rot_hi) {
            const double c2 = fma(2.0 * x2, x2, -1.0);
            const double s2 = dsqrt(1.0 - c2 * c2);
            const bool neg = rot_lo ? (x2 < 0.0 && x2 > -1.0) : (x2 > 0.0 && x2 < 1.0);
            c = c2;
            s = neg ? -s2 : s2;
        }
        so[0] = q[0];
        so[1] = c * q[1] + s * q[2];
        so[2] = -s * q[1] + c * q[2];
        so[3] = q[3];
        const double po = dsqrt(so[1] * so[1] + so[2] * so[2] + so[3] * so[3]);
        norm = (po > 0.0) ? dsqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]) / po : 1.0;
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

// the same with the first rotation given by its angle beta (mueller(beta) computed here unless
// HAVE_CS: the scattering path's sample_angles computed it for the same beta)
template <bool HAVE_CS = false>
__device__ __forceinline__ void polarization_rotation(const DevRun& R, double alpha, double beta, const double si[4],
                                                      const double sc[16], double d2, double dn2, double so[4], bool peeling,
                                                      double c2b = 0.0, double s2b = 0.0) {
    if constexpr (!HAVE_CS) mueller(beta, c2b, s2b);
    polarization_rotation_cs(R, alpha, c2b, s2b, beta >= 0.0 && beta < PI, beta >= PI && beta < TWO_PI, si, sc, d2, dn2, so,
                             peeling);
}

// The peel-off's polarization rotation (ARTES.f90:4864-4920): the Stokes vector st scattered
// by the interpolated matrix sc towards the detector (mu = cos of the scattering angle), in
// so[]; false when the reference skips the contribution (error 45) or drops the packet
// (error 49, `drop`).  (cpo, spo) is the incoming direction's azimuth (azimuth_cs).
// The rotation angle phs = acos(num), or its clamps 1e-10 / pi - 1e-10 (0 for a NaN), turned
// to 2 pi - phs when (phi_old - phi_det) mod 2 pi lies in [0, pi), enters polarization_rotation
// only through mueller(phs) and its half-turn: cos(2 phs) = 2 x^2 - 1 (x = num, or +-1 at
// the clamps, where the reference's cos(2 phs) rounds to 1), the sine negative on phs in
// (pi/2, pi) (x < 0) and on (3 pi/2, 2 pi) (turned, x > 0); no acos and no cosine.  The
// turn is decided from the azimuths' cosines and sines: sin(phi_old - phi_det) > 0, or the
// azimuths equal.  Where the difference is within rounding of 0 or pi the two forms can
// decide the turn differently.  There the direction, the detector and z lie in one plane,
// num = +-1 and sin(2 phs) ~ 0, so either turn gives the same vector -- unless the direction
// is within ~1e-6 rad of vertical, where num (through sqrt(1 - dz^2)) carries a relative
// error up to ~1e-4 in both forms and the turn is a rounding decision in the reference too
// (tests/test_gpu_unit_checks.py accepts either turn there, and checks every other case to
// 1e-7).
__device__ __forceinline__ bool peel_rotation(const DevRun& R, double dz, double mu, double cpo, double spo,
                                              const double st[4], const double sc[16], double so[4], bool& drop) {
    if (!(fabs(dz) < 1.0)) {
        log_err(R, 45);
        return false;
    }
    double num;
    {   // (the reference's evaluation, as direction_cosine_cs's num)
#pragma clang fp contract(off)
        num = (R.det2 - dz * mu) / (ref_sqrt(1.0 - mu * mu) * ref_sqrt(1.0 - dz * dz));
    }
    double x = 1.0;
    bool nan = false;
    if (fabs(num) < 1.0) x = num;
    else if (num >= 1.0) x = 1.0;
    else if (num <= -1.0) x = -1.0;
    else { log_err(R, 44); nan = true; }
    // (phi_old - phi_det) mod 2 pi in [0, pi): its sine > 0, or the azimuths equal
    const double sd = spo * R.cdphi - cpo * R.sdphi, cd = cpo * R.cdphi + spo * R.sdphi;
    const bool flip = sd > 0.0 || (sd == 0.0 && cd > 0.0);
    const double c2p = fma(2.0 * x, x, -1.0);
    double s2p = dsqrt(1.0 - c2p * c2p);
    if (flip ? (x > 0.0 && !nan) : (x < 0.0)) s2p = -s2p;
    if (!(fabs(mu) < 1.0)) {
        log_err(R, 49);
        drop = true;
        return false;
    }
    polarization_rotation_cs(R, mu, c2p, s2p, !flip, flip && !nan, st, sc, dz, R.det2, so, true);
    return true;
}

// the azimuth of direction (d0, d1) in [0, 2 pi) as direction_cosine takes it (ARTES.f90:1975-1977)
__device__ __forceinline__ double azimuth(double d0, double d1) {
    double phi = atan2(d1, d0);
    if (phi < 0.0) phi += TWO_PI;
    return phi;
}
// its cosine and sine without the angle: (d0, d1) / |(d0, d1)|, and (1, 0) for d0 = d1 = 0
// (atan2(0, 0) = 0)
__device__ __forceinline__ void azimuth_cs(double d0, double d1, double& c, double& s) {
    const double rho = dsqrt(d0 * d0 + d1 * d1);
    const double inv = rho > 0.0 ? 1.0 / rho : 0.0;
    c = rho > 0.0 ? d0 * inv : 1.0;
    s = d1 * inv;
}

// direction_cosine (ARTES.f90:1962-2052) with the old direction's azimuth given as its
// cosine and sine (cpo, spo).  The new azimuth phi_old -+ acos(num) is used only through
// its cosine and sine (2030-2050), so they follow from the angle-sum rule with
// cos(acos(num)) = num and sin(acos(num)) = sqrt(1 - num^2) >= 0: no atan2, acos or cosine
// of the angle.  The reference takes the sine as +-sqrt(1 - cos^2) by phi_new's half-turn,
// the same value up to rounding (its sign is sin(phi_new)'s); the error paths keep their
// phi_new = 0, i.e. (cos, sin) = (1, 0).
//
// The clamp of num at +-1 moves the azimuth by acos(1 - 1e-10) = 1.4e-5 rad on one side of it,
// so which side num rounds to is a decision, not a rounding: where the new direction lies in
// the old one's meridian plane (beta = 0 or pi) num is +-1 in exact arithmetic.  num and the
// four values it is made of are therefore evaluated as the reference writes them -- its
// operation order, no fused multiply-adds, correctly rounded square roots and division -- so
// the device takes the reference's side of the clamp wherever its cosine of beta rounds alike
// (tests/test_gpu_unit_checks.py, the boundary cases).
__device__ void direction_cosine_cs(const DevRun& R, double alpha, double beta, double d0, double d1, double d2,
                                    double cpo, double spo, double& e0, double& e1, double& e2) {
    const bool upper = (beta >= PI && beta < TWO_PI);
    const bool lower = (beta >= 0.0 && beta < PI);
    // (one cosine of the branch's argument: the same value, no divergent pair)
    const double cbeta = cos_b(upper ? TWO_PI - beta : beta);
    double cto, sto, ctn = 0.0, stn, num;
    {
#pragma clang fp contract(off)
        cto = d2 / ref_sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        sto = ref_sqrt(1.0 - cto * cto);
        if (upper || lower) ctn = cto * alpha + sto * ref_sqrt(1.0 - alpha * alpha) * cbeta;
        stn = ref_sqrt(1.0 - ctn * ctn);
        num = (alpha - ctn * cto) / (stn * sto);
    }
    if (!(upper || lower)) log_err(R, 18);
    if (num >= 1.0) num = 1.0 - 1.e-10;
    else if (num <= -1.0) num = -1.0 + 1.e-10;
    double cpn = 1.0, spn = 0.0;
    if (fabs(num) <= 1.0) {
        if (upper || lower) {
            const double san = dsqrt(1.0 - num * num);
            const double sg = upper ? -san : san;   // phi_new = phi_old - acos(num) (upper), + (lower)
            cpn = cpo * num - spo * sg;
            spn = spo * num + cpo * sg;
        } else {
            log_err(R, 19);
        }
    } else {
        log_err(R, 20);
    }
    e0 = stn * cpn;
    e1 = stn * spn;
    e2 = ctn;
}

// the same with the azimuth computed here (or given as the angle phi_in, HAVE_PHI)
template <bool HAVE_PHI = false>
__device__ __forceinline__ void direction_cosine(const DevRun& R, double alpha, double beta, double d0, double d1, double d2,
                                                 double& e0, double& e1, double& e2, double phi_in = 0.0) {
    double cpo, spo;
    if constexpr (HAVE_PHI) {
        cpo = cos_b(phi_in);
        spo = sin_b(phi_in);
    } else {
        azimuth_cs(d0, d1, cpo, spo);
    }
    direction_cosine_cs(R, alpha, beta, d0, d1, d2, cpo, spo, e0, e1, e2);
}

// linear interpolation of the 16 elements at angle acos(mu) between bin centres
// (ARTES.f90:1448-1530, 4780-4862); P = [180][RS] of the cell's matrix (RS = 16, or 17
// in LDS: see k_event).  sym: the call's matrices all have the block-diagonal form of
// spheres and Rayleigh scattering, [[P11 P12 0 0] [P12 P11 0 0] [0 0 P33 P34] [0 0 -P34 P33]]
// (checked value by value on the host, wl_set), and P = [180][RS4] holds (P11, P12, P33, P34):
// 4 reads and 4 interpolations per row instead of 16, the same 16 values bit for bit
// (the duplicated elements interpolate identically, the zeros to +0, and -P34's
// interpolation is the exact negative of P34's).
template <int RS = 16, int RS4 = 4>
__device__ __forceinline__ void interp_matrix_deg(const double* __restrict__ P, bool sym, double deg, double sc[16]) {
    const int ideg = (int)deg;
    int up, lo;
    if (deg - (double)ideg > 0.5) { up = ideg + 2; lo = ideg + 1; }
    else { up = ideg + 1; lo = ideg; }
    if (sym) {
        double v[4];
        if (up == 1) {
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = P[i];
        } else if (lo == 180) {
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = P[179 * RS4 + i];
        } else {
            const double* x0 = P + (lo - 1) * RS4;
            const double* x1 = P + (up - 1) * RS4;
            const double f = deg - ((double)lo - 0.5);   // (the reference divides by y1 - y0 = 1: exact)
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = (x1[i] - x0[i]) * f + x0[i];
        }
        sc[0] = v[0]; sc[1] = v[1]; sc[2] = 0.0; sc[3] = 0.0;
        sc[4] = v[1]; sc[5] = v[0]; sc[6] = 0.0; sc[7] = 0.0;
        sc[8] = 0.0; sc[9] = 0.0; sc[10] = v[2]; sc[11] = v[3];
        sc[12] = 0.0; sc[13] = 0.0; sc[14] = -v[3]; sc[15] = v[2];
        return;
    }
    if (up == 1) {
#pragma unroll
        for (int i = 0; i < 16; i++) sc[i] = P[i];
    } else if (lo == 180) {
#pragma unroll
        for (int i = 0; i < 16; i++) sc[i] = P[179 * RS + i];
    } else {
        const double* x0 = P + (lo - 1) * RS;
        const double* x1 = P + (up - 1) * RS;
        const double f = deg - ((double)lo - 0.5);   // (the reference divides by y1 - y0 = 1: exact)
#pragma unroll
        for (int i = 0; i < 16; i++) sc[i] = (x1[i] - x0[i]) * f + x0[i];
    }
}

// the same at angle acos(mu) (ARTES.f90:1448-1450: the angle in degrees)
template <int RS = 16, int RS4 = 4>
__device__ __forceinline__ void interp_matrix(const double* __restrict__ P, bool sym, double acos_mu, double sc[16]) {
    interp_matrix_deg<RS, RS4>(P, sym, acos_mu * 180.0 / PI, sc);
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

// the same by a 4-ary search: three probes per level, issued together, so the chain of
// dependent table reads is 4 levels long instead of 8 (180 -> 45 -> 12 -> 3 -> 1 bins)
template <typename F>
__device__ __forceinline__ int cdf_search4(double s, F cdf) {
    int lo = 1, hi = 180;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (lo < hi) {
            const int n = hi - lo;
            const int m1 = lo + (n >> 2), m2 = lo + (n >> 1), m3 = lo + ((3 * n) >> 2);
            const bool b1 = cdf(m1) >= s, b2 = cdf(m2) >= s, b3 = cdf(m3) >= s;
            if (b1) hi = m1;
            else if (b2) { lo = m1 + 1; hi = m2; }
            else if (b3) { lo = m2 + 1; hi = m3; }
            else lo = m3 + 1;
        }
    }
    return lo;
}

// The cumulative tables' element (j, k) (entry j = 0..180, column k = 0..3): [181][4] in global
// memory (CS = 4); in LDS (CS = 5) entries padded to 5 doubles.  ARTES_CUM_LAYOUT (A/B builds,
// profiles/r06/ab/event_lds_layout_ab.txt): 1 the four columns as separate arrays of 182, 2 the
// padded entries at an XOR-swizzled row j ^ ((j >> 4) & 15) (192 rows).
#ifndef ARTES_CUM_LAYOUT
#define ARTES_CUM_LAYOUT 0
#endif
template <int CS>
__host__ __device__ __forceinline__ int cum_at(int j, int k) {
    if constexpr (CS == 4 || ARTES_CUM_LAYOUT == 0) return j * CS + k;
    else if constexpr (ARTES_CUM_LAYOUT == 1) return k * 182 + j;
    else return (j ^ ((j >> 4) & 15)) * CS + k;
}
// doubles per LDS cumulative table of the layout
constexpr int cum_lds_doubles() { return ARTES_CUM_LAYOUT == 1 ? 4 * 182 : ARTES_CUM_LAYOUT == 2 ? 192 * 5 : 181 * 5; }

// scattering_angle_sampling (ARTES.f90:1534-1661) by searching the cumulative tables;
// C = [181][CS] (CS = 4, or 5 in LDS: see k_event, cum_at)
template <int CS = 4>
__device__ void sample_angles(const DevGrid& G, const DevRun& R, const double* __restrict__ C, Rng& rng,
                              const double st[4], double& alpha, double& beta, double& c2b, double& s2b,
                              double* adeg_out = nullptr) {
    // azimuth: C_b(i) = i (p11 I + p14 V) + (p12 Q + p13 U) SC2(i) + (p12 U - p13 Q) SS2(i)
    const double p11 = C[cum_at<CS>(180, 0)], p12 = C[cum_at<CS>(180, 1)], p13 = C[cum_at<CS>(180, 2)], p14 = C[cum_at<CS>(180, 3)];
    const double u = p11 * st[0] + p14 * st[3];
    const double v = p12 * st[1] + p13 * st[2];
    const double w = p12 * st[2] - p13 * st[1];
    auto cb = [&](int i) { return (double)i * u + v * G.sc2[i] + w * G.ss2[i]; };
    double s = rng.uni() * cb(180);
#ifdef ARTES_SEARCH2
    int i = cdf_search(s, cb);
#else
    int i = cdf_search4(s, cb);
#endif
    double y0 = cb(i - 1), y1 = cb(i);
    beta = (s - y0) / (y1 - y0) + (double)(i - 1);
    beta = beta * PI / 180.0;
    if (rng.uni() > 0.5) beta = beta + PI;
    if (beta >= TWO_PI) beta = TWO_PI - 1.e-10;
    if (beta <= 0.0) beta = -TWO_PI + 1.e-10;
    mueller(beta, c2b, s2b);
    // polar: C_t(i) = I A1(i) + (c2b Q + s2b U) A2(i) + (c2b U - s2b Q) A3(i) + V A4(i)
    const double k0 = st[0], k1 = c2b * st[1] + s2b * st[2], k2 = c2b * st[2] - s2b * st[1], k3 = st[3];
    auto ct = [&](int j) {
        return k0 * C[cum_at<CS>(j, 0)] + k1 * C[cum_at<CS>(j, 1)] + k2 * C[cum_at<CS>(j, 2)] + k3 * C[cum_at<CS>(j, 3)];
    };
    s = rng.uni() * ct(180);
#ifdef ARTES_SEARCH2
    i = cdf_search(s, ct);
#else
    i = cdf_search4(s, ct);
#endif
    y0 = ct(i - 1);
    y1 = ct(i);
    const double adeg = (s - y0) / (y1 - y0) + (double)(i - 1);
    if (adeg_out) *adeg_out = adeg;
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


}  // namespace artes
