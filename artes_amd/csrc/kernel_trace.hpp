// kernel_trace.hpp -- k_trace, the hot loop of the event engine.
//
// Every trace of the reference -- first optical depth (ARTES.f90:625-656), propagation
// (689-778, 848-941) and peel-off (4739-4761) -- is a sequence of cell_face calls
// (2800-3470): from the current position, the distance to every face of the current
// cell (inner/outer sphere, inner/outer theta cone or the 90-degree plane, the two phi
// half-planes) and the nearest one wins.
//
// Along a straight trace the faces of a coordinate family do not change until the trace
// crosses a face of THAT family: crossing a phi face leaves the cell's radial shell and
// theta band, so their candidate crossings are still the ones found before.  This
// kernel therefore keeps, per family, the nearest face ahead (as a trace parameter t) in
// registers and, after each crossing, re-evaluates only the family that was crossed -- with the
// reference's own formulas, tolerances and same-face rules, from the current position.
// That is one pair of quadratics (spheres or cones) or one pair of plane intersections
// per step instead of four quadratics and three plane intersections.  The family to
// evaluate differs from lane to lane, so the evaluation is written once for all three
// (coefficients and operands are selected per lane, the arithmetic is shared): the wave
// executes one evaluation per step, not three.  A new trace evaluates its families one
// per step before it moves (radial, theta, phi), so set-up costs two extra steps and no
// divergent branch.
//
// Divisions and square roots use reciprocal / reciprocal-square-root seeds refined by
// Newton steps (<= 1-2 ulp); the reference's correctly rounded forms cost twice the VALU
// work, and the trajectory parity tests (tests/test_gpu_parity.py) bound the effect.
#pragma once

#include "device_common.hpp"

#ifdef ARTES_TWOFACE
static constexpr bool TWOFACE = true;    // A/B builds: evaluate both faces of every family
#else
static constexpr bool TWOFACE = false;
#endif
#ifdef ARTES_NO_TREL
static constexpr bool TREL_ON = false;   // A/B builds: the radial family re-solved from the current point
#else
static constexpr bool TREL_ON = true;    // the radial family trace-relative (radial_tr)
#endif
// ARTES_DEBUG_TIMING (development build, tools/time_regions.py): per wave, the shader-clock
// cycles spent in each region of the k_trace loop, summed into the error slots 0-7 (the
// run's error codes are void then)
#ifdef ARTES_DEBUG_TIMING
#define TM_TICK(v) const unsigned long long v = tm_tick()
#define TM_ADD(k, d) tm_add(k, d)
#else
#define TM_TICK(v)
#define TM_ADD(k, d)
#endif
#ifdef ARTES_LOOKAHEAD
static constexpr bool LOOKAHEAD = true;   // A/B builds: slot ids from the chunk registers, records prefetched (kernel_event.hpp)
#else
static constexpr bool LOOKAHEAD = false;   // refills load list entries and records on demand ("lookahead refills")
#endif

namespace artes {

// ------------------------------------------------------------ fast math ---
// a / b to ~1 ulp for normal operands (b = 0 gives inf/nan: callers select it away).
// v_rcp_f64 is good to ~2^-23; one Newton step squares that error, and the residual
// correction of the quotient squares it again, below the rounding of the result.
__device__ __forceinline__ double fast_div(double a, double b) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    const double q = a * r;
    return fma(fma(-b, q, a), r, q);
}
__device__ __forceinline__ double fast_rcp(double b) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    return fma(fma(-b, r, 1.0), r, r);
}
// sqrt(x) to ~1 ulp for x > 0 (x <= 0 gives 0)
__device__ __forceinline__ double fast_sqrt(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
    const double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    const double d = fma(-g, g, x);
    g = fma(d, h, g);
    return x > 0.0 ? g : 0.0;
}

// sqrt(x) to ~1 ulp for x >= 0 (x < 0: any value; callers reject those roots): the seed
// capped so that x = 0 gives 0 * 1e300 = 0 instead of 0 * inf.  (fmin, not an inline
// v_min: the compiler must see the transcendental's result being read, for gfx950's
// trans-use hazard wait.)
__device__ __forceinline__ double fast_sqrt0(double x, double cap = 1.e300) {
    const double y = fmin(__builtin_amdgcn_rsq(x), cap);
    double g = x * y, h = 0.5 * y;
    const double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    const double d = fma(-g, g, x);
    return fma(d, h, g);
}

// sqrt(x) to ~1 ulp for x > 0; NaN for x <= 0 (0 * rsq(0) = 0 * inf).  For the radial roots,
// where a zero or negative discriminant gives no crossing and NaN roots fail every test.
// (One Goldschmidt step takes the seed's ~2^-23 to ~2^-46; the correction g + d h then needs h
// only to the seed's accuracy -- its error multiplies d ~ 2^-46 g -- so h is not refined.)
__device__ __forceinline__ double fast_sqrt_nan0(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    const double h = 0.5 * y;
    const double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    const double d = fma(-g, g, x);
    return fma(d, h, g);
}

// The step's threshold constants in vector registers, loaded once per kernel.  gfx950's
// VOP3 compares and FMAs take no 64-bit literal, so a constant operand is two scalar moves
// at every use, and with machine LICM off (Makefile) every step rematerialises them; k_trace
// has vector registers to spare at 4 waves per SIMD on 3D grids (108 of 128), so there the
// thresholds live in them.  (The inline move makes them opaque: the compiler cannot fold them back.)
struct TraceK {
    double tiny, tol, tol_same, huge, cap, step_min, inf;   // 1e-100 1e-15 1e-3 1e100 1e300 1e-9 inf
    int nan_hi;                                             // 0x7FF80000: a quiet NaN's high word (or_nan)
};
__device__ __forceinline__ double vreg(double c) {
    double r;
    asm volatile("v_mov_b64 %0, %1" : "=v"(r) : "s"(c));
    return r;
}
__device__ __forceinline__ int vreg_i(int c) {
    int r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(c));
    return r;
}
template <bool IN_VGPRS>
__device__ __forceinline__ TraceK trace_consts() {
    if constexpr (IN_VGPRS)
        return TraceK{vreg(1.e-100), vreg(1.e-15), vreg(1.e-3), vreg(1.e100), vreg(1.e300), vreg(1.e-9), vreg(__builtin_inf()),
                      vreg_i(0x7FF80000)};
    else
        return TraceK{1.e-100, 1.e-15, 1.e-3, 1.e100, 1.e300, 1.e-9, __builtin_inf(), 0x7FF80000};
}

// ---------------------------------------------------- face tables (LDS) ---
// The spheres and the theta cones are one quadric form along the ray,
//     ax2 x^2 + by2 y^2 + w cz2 z^2 - off = 0,
// with (w, off) = (1, rfront^2) for a radial face and (-tan^2(theta_f), 0) for a theta
// face (ARTES.f90:2885-3010, 3014-3290).  A face record is {w, off, s, flags}: s is the
// cone's nappe sign (+1: theta_f > 90 deg, a root with z > 0 is on the other nappe;
// -1: theta_f < 90 deg, z < 0 is; 0: radial faces and the 90-degree plane); the flags
// hold the face's rules as bits, read instead of derived per lane (FR_*): the 90-degree
// plane (tplane = 2); the same-face veto when the packet sits on the face and it is the
// cell's outer (KS_OUT) or inner (KS_IN) face -- a sphere only as the inner face
// (ARTES.f90:2899-2960), a cone when it is the plane or the packet is on the far side of
// its apex (3014-3290); the grid's polar theta faces, never crossed (EDGE); the 1e-3 m
// same-face tolerance as outer / inner face (a sphere only as the outer face, a cone
// both; 2944, 3157).  The records of the radial faces 0..nr are followed by those of the
// theta faces 0..ntheta, so every family reads its faces with the same instructions and
// no per-lane select of coefficients or flags (the phi family reads radial records, and
// ignores them); phsc[k] = (sin, cos)(phi_k).
struct alignas(32) FaceRec {
    double w, off, s;
    int flags, pad;
};
enum : int { FR_PL = 1, FR_KS_OUT = 2, FR_KS_IN = 4, FR_EDGE = 8, FR_BIG_OUT = 16, FR_BIG_IN = 32 };

struct TraceTabs {
    const FaceRec* fr;
    const double2* phsc;
    const double2* tcs;   // (cos, sin)(theta_k), for the set-up bounds
    const double2* rr;    // (r_k, r_k+1): a radial shell's two radii (the trace-relative sphere roots)
};

// (rr has nr + 1 entries: the fused radial step reads rr[kn] for kn = -1 .. nr before it knows
// whether the packet stays in the grid -- rr[-1] is the last tcs entry, rr[nr] a pad -- and uses
// the values only when kn names a shell)
__host__ __device__ inline size_t trace_table_bytes(int nr, int ntheta, int nphi) {
    return sizeof(FaceRec) * ((size_t)(nr + 1) + (size_t)(ntheta + 1)) + sizeof(double2) * ((size_t)nphi + ntheta + 1 + nr + 1);
}
// The tables' layout from `base` (LDS, or the global copy of the GTAB kernels)
__device__ __forceinline__ TraceTabs trace_tables_at(const DevGrid& G, double* base) {
    TraceTabs T;
    FaceRec* fr = (FaceRec*)base;
    double2* phsc = (double2*)(fr + (G.nr + 1) + (G.ntheta + 1));
    double2* tcs = phsc + G.nphi;
    double2* rr = tcs + G.ntheta + 1;
    T.fr = fr; T.phsc = phsc; T.tcs = tcs; T.rr = rr;
    return T;
}
// Fill the tables at `base`, thread `tid` of `nt`
__device__ __forceinline__ void fill_trace_tables(const DevGrid& G, double* base, int tid, int nt) {
    const TraceTabs T = trace_tables_at(G, base);
    FaceRec* fr = (FaceRec*)T.fr;
    for (int i = tid; i <= G.nr; i += nt) fr[i] = FaceRec{1.0, G.rf2[i], 0.0, FR_KS_IN | FR_BIG_OUT, 0};
    for (int i = tid; i <= G.ntheta; i += nt) {
        const double th = G.thetaf[i];
        const bool cone = G.tplane[i] == 1;
        const double sg = cone ? (th > HALF_PI ? 1.0 : (th < HALF_PI ? -1.0 : 0.0)) : 0.0;
        const int fl = (cone ? 0 : FR_PL) | ((!cone || !(sg < 0.0)) ? FR_KS_OUT : 0) | ((!cone || !(sg > 0.0)) ? FR_KS_IN : 0) |
                       ((i == 0 || i == G.ntheta) ? FR_EDGE : 0) | FR_BIG_OUT | FR_BIG_IN;
        fr[G.nr + 1 + i] = FaceRec{-G.tan2[i], 0.0, sg, fl, 0};
    }
    double2* phsc = (double2*)T.phsc;
    for (int i = tid; i < G.nphi; i += nt) phsc[i] = make_double2(G.phis[i], G.phic[i]);
    double2* tcs = (double2*)T.tcs;
    for (int i = tid; i <= G.ntheta; i += nt) {
        const double c = G.tcos[i];
        tcs[i] = make_double2(c, sqrt(fmax(0.0, 1.0 - c * c)));
    }
    double2* rr = (double2*)T.rr;
    for (int i = tid; i <= G.nr; i += nt) rr[i] = make_double2(G.rfr[i], G.rfr[i < G.nr ? i + 1 : i]);
}
// The tables in LDS, staged by the block
__device__ __forceinline__ TraceTabs stage_trace_tables(const DevGrid& G, double* lds) {
    fill_trace_tables(G, lds, threadIdx.x, BLOCK);
    __syncthreads();
    return trace_tables_at(G, lds);
}

// The global copy of the GTAB kernels (one block, once per call before the engine loop): grids
// whose tables exceed the 64 KiB k_trace stages in LDS (e.g. a fine P-T gas profile of ~2000
// radial faces; the reference allocates any grid, ARTES.f90:2237-2307) read them from L2
__global__ __launch_bounds__(BLOCK) void k_fill_trace_tables(DevGrid G) { fill_trace_tables(G, G.ttab, threadIdx.x, BLOCK); }

// min of two doubles, one v_min_f64 without the canonicalising v_max the IEEE-mode fmin
// needs on unknown operands.  A quiet-NaN operand (or_nan below: "no crossing") yields the
// other operand (IEEE minNum); two NaNs yield a NaN.  Its operands must not be the direct
// result of a transcendental (v_rcp / v_rsq / v_exp ...): the compiler does not insert the
// gfx950 trans-use hazard wait before inline assembly.
__device__ __forceinline__ double min_nonan(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

constexpr double INF = __builtin_inf();

// k_trace's face the packet sits on, as one code: (type - 1) << 16 | index for a radial (type 1),
// theta (2) or phi (3) face -- a radial face's code is its index -- and -1 for none (type 0).
// One register instead of two, and "on sphere k" is one compare (the record keeps pack_face's
// form; the event engine's cell packing keeps every index <= 4096, transport.hip)
__device__ __forceinline__ int face_code(int type, int idx) { return type == 0 ? -1 : ((type - 1) << 16) | idx; }
__device__ __forceinline__ int face_code_type(int tf) { return (tf >> 16) + 1; }   // (arithmetic shift: -1 -> 0)
__device__ __forceinline__ int face_code_index(int tf) { return tf < 0 ? 0 : (tf & 0xFFFF); }

// k_trace's `parked` codes: 1 (3 after a cell error) the forced first interaction waits, 4 the
// interaction waits; PK_END and its bits (trace-relative kernels): a trace end found in a step,
// resolved at the end of the iteration
// PK_RAD: a trace end of the radial-form step, whose exit / surface / runaway bits the end block
// derives from the state (tf the sphere crossed, ncross against nlim) instead of the step; its
// codes PK_RAD_END and PK_RAD_ERR are inline constants of the instruction set (<= 64), so the step
// selects them with no literal moves (bits 0-1 of a code >= PK_END are free: the parked-lane
// tests of the loop head see codes 1, 3, 4 only)
enum : int { PK_END = 8, PK_EXIT = 16, PK_SURF = 32, PK_ERR31 = 64, PK_RUNAWAY = 128, PK_ERR = 256, PK_RAD = 1, PK_RAD_E = 2 };
enum : int { PK_RAD_END = PK_END | PK_RAD, PK_RAD_ERR = PK_END | PK_RAD | PK_RAD_E };
// a new trace's set-up (k_trace's common set-up block): the start cell from the packet position,
// the direction's constants
enum : int { NT_POS = 1, NT_DIR = 2 };

// x if valid, else a NaN: only the high word is selected (one v_cndmask instead of two
// for a double select).  min_nonan ignores the NaN, and every compare with it is false, so
// a NaN distance means "no crossing" as +inf does.
__device__ __forceinline__ double or_nan(bool valid, double x) {
    return __hiloint2double(valid ? __double2hiint(x) : 0x7FF80000, __double2loint(x));
}
// the same with the NaN's high word from a register (gfx950's VOP3 select takes no literal)
__device__ __forceinline__ double or_nan(bool valid, double x, int nan_hi) {
    return __hiloint2double(valid ? __double2hiint(x) : nan_hi, __double2loint(x));
}

// the scaled squared length of a direction's xy part (one expression for every caller, so
// a constant computed once rounds as the per-trace one would)
__device__ __forceinline__ double dir_axy(double ax2, double by2, double d0, double d1) { return ax2 * d0 * d0 + by2 * d1 * d1; }

// ------------------------------------------------------- family evaluation ---
// Nearest crossing ahead among the inner and outer face of ONE coordinate family of cell
// (cr, ct, cp) from (x, y, z) along n, for a packet sitting on face (ft, fi):
//   fam 0: spheres r_cr, r_cr+1   (ARTES.f90:2885-3010)
//   fam 1: theta cones / the 90-degree plane, faces ct, ct+1 (3014-3290)
//   fam 2: phi half-planes cp, pout (3292-3350)
// Returns the distance (+inf: no candidate) and whether it is the outer face.  zp = the
// distance to the plane z = 0; Axy = ax2 n0^2 + by2 n1^2, Az = cz2 n2^2 (per trace).
//
// Per face k (0 inner, 1 outer) the reference's rules reduce to: two roots a_k, b_k
// (phi planes and the 90-degree plane: one), each a candidate when it exists, lies on the
// right nappe (cones), exceeds the face's tolerance and is < 1e100; none when both exist
// and are equal, or when a per-face veto (same-face and grid-edge rules) applies; the
// nearer candidate wins (quadratic_equation + cell_face root choice, ARTES.f90:2885-3350,
// 4154-4173).  Absent candidates are +inf, so the choice is one min.  The 1e100 cap of
// the chosen root is applied per root: the nearer root of a pair is below 1e100 iff
// the reference's choice is.  A root exists when its divisor exceeds 1e-100 in
// magnitude (the reference's |den| > 0 for the phi planes differs only where num/den is
// >= 1e100 anyway; the sp0 quirk keeps |den| > 0).  The conditions are written as
// monotone AND/OR of comparisons (no selects of booleans), which stay lane masks.
template <bool G3D, bool OBL>
__device__ __forceinline__ double family_eval(const DevGrid& G, const TraceTabs& T, int fam, double x, double y, double z,
                                              double n0, double n1, double n2, double Axy, double Az, int tf,
                                              int cr, int ct, int cp, int pout, double zp, bool& outer) {
    const double ax2 = OBL ? G.ax2 : 1.0, by2 = OBL ? G.by2 : 1.0, cz2 = OBL ? G.cz2 : 1.0;
    [[maybe_unused]] const bool isR = !G3D || fam == 0;
    const bool isT = G3D && fam == 1;
    const bool isP = G3D && fam == 2;
    const double Bxy = ax2 * x * n0 + by2 * y * n1, Bz = cz2 * z * n2;
    const double Cxy = ax2 * x * x + by2 * y * y, Cz = cz2 * z * z;
    const int kin = isT ? ct : cr;
    const int e = (isT ? G.nr + 1 : 0) + kin;
    const FaceRec fin = T.fr[e], fout = T.fr[e + 1];
    // radial-only grids: w = 1 (spheres only), no nappe sign, no plane
    const double w0 = G3D ? fin.w : 1.0, w1 = G3D ? fout.w : 1.0;
    const double s0 = G3D ? fin.s : 0.0, s1 = G3D ? fout.s : 0.0;
    const double qa0 = fma(w0, Az, Axy), qb0 = 2.0 * fma(w0, Bz, Bxy), qc0 = fma(w0, Cz, Cxy) - fin.off;
    const double qa1 = fma(w1, Az, Axy), qb1 = 2.0 * fma(w1, Bz, Bxy), qc1 = fma(w1, Cz, Cxy) - fout.off;
    // quadratic_equation (ARTES.f90:4154-4173), both faces
    const double disc0 = qb0 * qb0 - 4.0 * qa0 * qc0, disc1 = qb1 * qb1 - 4.0 * qa1 * qc1;
    const double q0 = -0.5 * (qb0 + copysign(fast_sqrt(disc0), qb0));
    const double q1 = -0.5 * (qb1 + copysign(fast_sqrt(disc1), qb1));
    // phi half-planes: num / den per face (ARTES.f90:3300-3346)
    double num0 = 0.0, den0 = 1.0, num1 = 0.0, den1 = 1.0;
    if constexpr (G3D) {
        const double ga = OBL ? G.a : 1.0, gb = OBL ? G.b : 1.0;
        const double2 sc0 = T.phsc[cp], sc1 = T.phsc[pout];
        den0 = gb * n1 * sc0.y - ga * n0 * sc0.x; num0 = ga * x * sc0.x - gb * y * sc0.y;
        den1 = gb * n1 * sc1.y - ga * n0 * sc1.x; num1 = ga * x * sc1.x - gb * y * sc1.y;
    }
    // four divisions shared by the families: the roots q/a and c/q, or the plane
    // intersections num/den
    const double da0 = isP ? den0 : qa0, da1 = isP ? den1 : qa1;
    const double a0r = fast_div(isP ? num0 : q0, da0);
    const double b0 = fast_div(qc0, q0);
    const double a1r = fast_div(isP ? num1 : q1, da1);
    const double b1 = fast_div(qc1, q1);
    const int kout = kin + 1;
    const int kin_f = isP ? cp : kin, kout_f = isP ? pout : kout;
    const int fb = fam << 16;   // (the face code, see face_code)
    const bool same0 = tf == kin_f + fb, same1 = tf == kout_f + fb;
    const bool plane0 = G3D && (fin.flags & FR_PL), plane1 = G3D && (fout.flags & FR_PL);   // (theta lanes only)
    // existence: the divisor, and for the quadratic the discriminant
    const bool d_ok0 = isP | (disc0 >= 0.0), d_ok1 = isP | (disc1 >= 0.0);
    bool va0 = d_ok0 & (fabs(da0) > 1.e-100);
    bool vb0 = !isP & (disc0 >= 0.0) & (fabs(q0) > 1.e-100);
    bool va1 = d_ok1 & (fabs(da1) > 1.e-100);
    bool vb1 = !isP & (disc1 >= 0.0) & (fabs(q1) > 1.e-100);
    // cone nappe filter (ARTES.f90:3040-3064): a root on the other nappe is no crossing;
    // s = 0 (radial records, the plane) never rejects
    if constexpr (G3D) {
        va0 = va0 & !(s0 * fma(a0r, n2, z) > 0.0);
        vb0 = vb0 & !(s0 * fma(b0, n2, z) > 0.0);
        va1 = va1 & !(s1 * fma(a1r, n2, z) > 0.0);
        vb1 = vb1 & !(s1 * fma(b1, n2, z) > 0.0);
    }
    // tolerances: re-crossing the face the packet sits on needs 1e-3 m (spheres: outer
    // face only, cones: both; ARTES.f90:2944, 3157), 1e-15 otherwise; the 90-degree plane
    // has one root at zp, valid when moving towards it (ARTES.f90:3066-3070, 3116-3118)
    const bool big0 = same0 & isT, big1 = same1 & !isP;
    const double a0 = plane0 ? zp : a0r, a1 = plane1 ? zp : a1r;
    va0 = (va0 & !plane0 & (a0 > 1.e-15) & (!big0 | (a0 > 1.e-3))) | (plane0 & (n2 > 1.e-15) & (a0 > 0.0));
    va1 = (va1 & !plane1 & (a1 > 1.e-15) & (!big1 | (a1 > 1.e-3))) | (plane1 & (n2 < -1.e-15) & (a1 > 0.0));
    vb0 = vb0 & !plane0 & (b0 > 1.e-15) & (!big0 | (b0 > 1.e-3));
    vb1 = vb1 & !plane1 & (b1 > 1.e-15) & (!big1 | (b1 > 1.e-3));
    // vetoes
    //   spheres: the inner sphere the packet sits on (ARTES.f90:2899-2960)
    //   theta:   the grid's polar faces; a cone the packet sits on unless the root lies
    //            beyond the apex side it faces; the plane it sits on (3014-3290)
    //   phi:     the half-plane the packet sits on; the outer one also when the inner
    //            face's root is >= 1e100 (sic: sp0, ARTES.f90:3318, 3346)
    const bool kill0 = (same0 & !isT) | (isT & ((ct == 0) | (same0 & (plane0 | !(s0 > 0.0)))));
    const bool sp0_big = isP & !same0 & (fabs(den0) > 0.0) & !(a0r < 1.e100);
    const bool kill1 = (isT & ((kout == G.ntheta) | (same1 & (plane1 | !(s1 < 0.0))))) | (isP & same1) | sp0_big;
    // equal roots give no crossing; the 1e100 cap
    const bool eq0 = va0 & vb0 & (a0 == b0), eq1 = va1 & vb1 & (a1 == b1);
    va0 = va0 & !kill0 & !eq0 & (a0 < 1.e100);
    vb0 = vb0 & !kill0 & !eq0 & (b0 < 1.e100);
    va1 = va1 & !kill1 & !eq1 & (a1 < 1.e100);
    vb1 = vb1 & !kill1 & !eq1 & (b1 < 1.e100);
    const double m0 = min_nonan(va0 ? a0 : INF, vb0 ? b0 : INF);
    const double m1 = min_nonan(va1 ? a1 : INF, vb1 ? b1 : INF);
    outer = m1 < m0;   // ties: the inner face, as the reference's candidate order
    return min_nonan(m0, m1);
}

// ------------------------------------------------ one-face family evaluation ---
// The face of a radial shell or theta band that a straight ray can cross NEXT is known
// before any root is computed:
//  * spheres: |p(t)|^2 is convex along the ray.  Moving inwards (p.n < 0) with the ray
//    reaching the inner sphere (discriminant >= 0), the inner crossing comes first (both
//    its roots lie ahead, before the perigee, and the outer sphere is only left after
//    it); otherwise the outer sphere.  The inner sphere the packet sits on is never a
//    candidate (ARTES.f90:2899-2960), so that case is the outer sphere too.
//  * theta cones: a line meets any cone level at most twice, so theta(t) has at most one
//    extremum: the face in the direction theta moves (d cos(theta)/dt ~ n2 C - z B) is the
//    next one if it is crossed at all; if theta turns back first, that face has no valid
//    root and the other face is evaluated in the lane's next iteration (`alt`, at most
//    once per trace).  The same fallback covers the sphere's degenerate cases (a double
//    root) exactly.
//  * phi half-planes: both faces, as before (cheap, and the sp0 quirk needs the inner one).
// So a family costs one quadratic (one square root) instead of two, and the same rules as
// family_eval's apply to the two roots of the chosen face (for phi: one root per face).
//
// NORAD: the caller evaluates the radial family elsewhere (radial_tr), so fam is 1 or 2
// here: the sphere's face choice folds away.
template <bool G3D, bool OBL, bool NORAD = false>
__device__ __forceinline__ double family_eval1(const DevGrid& G, const TraceTabs& T, int fam, double x, double y, double z,
                                               double n0, double n1, double n2, double Axy, double Az, int tf,
                                               int cr, int ct, int cp, int pout, double zp, bool alt, const TraceK& K,
                                               bool& outer) {
    const double ax2 = OBL ? G.ax2 : 1.0, by2 = OBL ? G.by2 : 1.0, cz2 = OBL ? G.cz2 : 1.0;
    const bool isT = G3D && (NORAD ? fam != 2 : fam == 1);
    const bool isP = G3D && fam == 2;
    const double Bxy = ax2 * x * n0 + by2 * y * n1, Bz = cz2 * z * n2;
    const double Cxy = ax2 * x * x + by2 * y * y, Cz = cz2 * z * z;
    const int kin = isT ? ct : cr;
    const int e = (isT ? G.nr + 1 : 0) + kin;
    const int fb = fam << 16;   // (the face code, see face_code)
    const bool same_in = tf == (isP ? cp : kin) + fb;
    // which face: the sphere rule needs the inner face's discriminant (w = 1)
    bool ch;
    if constexpr (NORAD) {   // theta: the face theta moves to; phi: (unused)
        const bool t_out = fma(n2, Cxy + Cz, -z * (Bxy + Bz)) < 0.0;
        ch = (isT & t_out) != alt;
    } else {
        const double off_in = T.fr[e].off;
        const double qa_in = Axy + Az, hb = Bxy + Bz, qc_in = Cxy + Cz - off_in;
        // (the discriminant exactly as the roots below compute it for this face: written
        // as a plain hb*hb - qa*qc the compiler contracts it into an FMA of its own choosing,
        // and a grazing ray could then see the inner sphere here but not there, or back)
        const bool in_ok = (hb < 0.0) & (fma(hb, hb, -(qa_in * qc_in)) >= 0.0) & !same_in;
        const bool t_out = fma(n2, Cxy + Cz, -z * hb) < 0.0;
        ch = (isT & t_out) | (!isT & !in_ok);   // (as masks: no branch around the radial record's read)
        ch = ch != alt;
    }
    const FaceRec fc = T.fr[e + (ch ? 1 : 0)];
    const double w = G3D ? fc.w : 1.0, sg = G3D ? fc.s : 0.0;
    const int fl = G3D ? fc.flags : (FR_KS_IN | FR_BIG_OUT);
    const bool pl = G3D && (fl & FR_PL);
    // quadratic_equation (ARTES.f90:4154-4173) in the half-b form: with qb = 2 hb the
    // reference's disc = qb^2 - 4 qa qc and q = -(qb + sign(qb) sqrt(disc)) / 2 are exactly
    // 4 disc4 and -(hb + sign(hb) sqrt(disc4)) (power-of-two scalings round alike)
    const double qa = fma(w, Az, Axy), hb = fma(w, Bz, Bxy), qc = fma(w, Cz, Cxy) - fc.off;
    const double disc = fma(hb, hb, -(qa * qc));
    const double q = -(hb + copysign(fast_sqrt0(disc, K.cap), hb));
    double num0 = 0.0, den0 = 1.0, num1 = 0.0, den1 = 1.0;
    if constexpr (G3D) {
        const double ga = OBL ? G.a : 1.0, gb = OBL ? G.b : 1.0;
        const double2 sc0 = T.phsc[cp], sc1 = T.phsc[pout];
        den0 = gb * n1 * sc0.y - ga * n0 * sc0.x; num0 = ga * x * sc0.x - gb * y * sc0.y;
        den1 = gb * n1 * sc1.y - ga * n0 * sc1.x; num1 = ga * x * sc1.x - gb * y * sc1.y;
    }
    // root A: the quadratic's q/a, or phi face 0; root B: c/q, or phi face 1
    const double dA = isP ? den0 : qa, dB = isP ? den1 : q;
    const double rA = fast_div(isP ? num0 : q, dA);
    const double rB = fast_div(isP ? num1 : qc, dB);
    const int kA = isP ? cp : kin + (ch ? 1 : 0), kB = isP ? pout : kA;
    const bool sameA = tf == kA + fb, sameB = tf == kB + fb;
    // existence: the divisor, and for the quadratic the discriminant
    const bool d_ok = isP | (disc >= 0.0);
    bool vA = d_ok & (fabs(dA) > K.tiny);
    bool vB = d_ok & (fabs(dB) > K.tiny);
    // cone nappe filter (ARTES.f90:3040-3064); sg = 0 never rejects
    if constexpr (G3D) {
        vA = vA & !(sg * fma(rA, n2, z) > 0.0);
        vB = vB & !(sg * fma(rB, n2, z) > 0.0);
    }
    // tolerances (1e-3 m to re-cross the face the packet sits on: spheres outer face only,
    // cones both; ARTES.f90:2944, 3157); the 90-degree plane: one root at zp, valid when
    // moving towards it (3066-3070, 3116-3118)
    // (the chosen face's rules as outer (ch) or inner face: flag bits 1 / 2 and 4 / 5; a
    // quadratic's two roots are on one face, so they share them)
    // (one AND of the flags with the bits that apply -- the role's two when the packet sits
    // on the face, the edge bit always -- then a test per rule: integer selects of constants,
    // where per-rule bit extractions cost lane-mask/VGPR conversions)
    // (radial-only grids: the sphere's rules, 1e-3 m as outer face, the veto as inner face)
    const int fsel = (sameA & !isP) ? (ch ? (FR_KS_OUT | FR_BIG_OUT) : (FR_KS_IN | FR_BIG_IN)) : 0;
    const int fhit = fl & (fsel | FR_EDGE);
    const double A = pl ? zp : rA;
    const bool big = G3D ? (fhit & (FR_BIG_OUT | FR_BIG_IN)) != 0 : sameA & ch;
    const double n2s = ch ? -n2 : n2;   // (moving towards the plane: n2 < 0 as outer face, > 0 as inner)
    const double tmin = big ? K.tol_same : K.tol;   // (one threshold per lane: two compares fewer in the mask logic)
    vA = (vA & !pl & (A > tmin)) | (pl & (n2s > K.tol) & (A > 0.0));
    vB = vB & !pl & (rB > tmin);
    // vetoes (ARTES.f90:2899-2960, 3014-3290, 3318, 3346)
    const bool qkill = G3D ? (fhit & (FR_EDGE | FR_KS_OUT | FR_KS_IN)) != 0 : sameA & !ch;
    const bool sp0_big = !sameA & (fabs(den0) > 0.0) & !(rA < K.huge);
    const bool killA = isP ? sameA : qkill;
    const bool killB = isP ? (sameB | sp0_big) : qkill;
    // equal roots of a quadratic give no crossing; the 1e100 cap
    const bool eq = !isP & vA & vB & (A == rB);
    vA = vA & !killA & !eq & (A < K.huge);
    vB = vB & !killB & !eq & (rB < K.huge);
    outer = isP ? (vB & (!vA | (rB < A))) : ch;
    return min_nonan(or_nan(vA, A), or_nan(vB, rB));   // NaN: no crossing
}

// ------------------------------------------- radial family, trace-relative (TREL) ---
// The radial faces take ~99.9 % of all crossings on the bench grid and 99.6 % on the
// configs[3] cloudy grid (their theta and phi cells are 1e3-1e4 times wider than a radial
// shell), and along the trace p(s) = p0 + s n the spheres' crossings are known from two
// per-trace numbers: b0 = p0.n and the perigee distance pm = |p0 x n|.  Sphere r meets the
// trace at s = -b0 -+ sqrt((r - pm)(r + pm)) (|n| = 1 to rounding), so an evaluation is one
// square root and no division, from the trace's start instead of the current point.  The
// factored discriminant keeps grazing rays accurate: r^2 - pm^2 at 5e15 m^2 would lose the
// millimetres near tangency that (r - pm)(r + pm) keeps.  The reference's rules follow with
// the distances from the current point, s - t (ARTES.f90:2885-3010): the face the trace
// can cross next (the inner sphere when moving inwards -- t before the perigee -- the ray
// reaches it, and the packet does not sit on it; else the outer one; `alt` the other one
// after a miss), re-crossing the sphere the packet sits on needs 1e-3 m as the outer face and
// is vetoed as the inner face, 1e-15 m otherwise, equal roots and >= 1e100 give none.
// Returns the crossing's trace parameter s (a NaN: none).  The roots differ from the
// reference's per-step re-solve by rounding (~1e-8 m at 7e7 m); the trajectory tests bound it.
__device__ __forceinline__ double radial_tr(const TraceTabs& T, double b0, double pm, double t, int tf, int cr,
                                            bool alt, const TraceK& K, bool& outer) {
    const double2 rr = T.rr[cr];
    // the packet sits on the shell's inner / outer sphere (a radial face's code is its index)
    const bool s_in = tf == cr, s_out = tf == cr + 1;
    const bool in_ok = (t < -b0) & (rr.x >= pm) & !s_in;
    const bool ch = in_ok == alt;   // outer face: !in_ok, turned by alt
    const double r = ch ? rr.y : rr.x;
    const double disc = (r - pm) * (r + pm);
    // (no cap on the rsq seed: a zero discriminant -- a double root, which gives no crossing --
    // then yields NaN roots, and a negative one NaN as well; every comparison of a NaN is false,
    // so both roots are rejected exactly as by the reference's rules; two instructions and the
    // discriminant's test fewer than fast_sqrt0)
    const double sq = fast_sqrt_nan0(disc);
    const double sA = -b0 - sq, sB = sq - b0;
    const double dA = sA - t, dB = sB - t;
    // (re-crossing the sphere the packet sits on: 1e-3 m as the outer face, vetoed as the inner one)
    const double tmin = (ch & s_out) ? K.tol_same : K.tol;
    // (equal roots give none: with dA == dB both pass or fail their tests together, so the
    // rule is one more term of each AND chain; the chains stay lane masks, and the nearer
    // valid root is one min -- sA <= sB -- instead of a branch)
    const bool ok = !(!ch & s_in) & (dA != dB);
    const bool vA = ok & (dA > tmin) & (dA < K.huge), vB = ok & (dB > tmin) & (dB < K.huge);
    outer = ch;
    return min_nonan(or_nan(vA, sA), or_nan(vB, sB));
}

// The radial family right after a sphere crossing, inside the radial-form step (the fused
// step, k_trace): radial_tr for a packet on face (1, nfi) of its new shell `rr` -- on the
// shell's inner sphere after an outward crossing (s_in = side), on its outer one after an
// inward crossing (s_out = !side) -- with alt = false (a lane steps radially only with its
// alt bit clear).  Within a monotone run of the trace the rules resolve the same way every
// time: inwards the inner sphere's near root sA while the ray reaches it, outwards the outer
// sphere's far root sB, and at the turn (the ray misses the inner sphere) the far root of the
// sphere just crossed, at 1e-3 m (ARTES.f90:2885-3010).  The same operations in the same order
// as radial_tr, so the same bits; only the two face tests are known from the step's side.
// The 1e100 caps of radial_tr are left out: the roots and the trace parameter lie within 4 r_top
// of the trace's start, and grids are limited to r_top < 1e40 m (artes_grid_create).
// A NaN (no crossing: the other face next, `alt`) sends the lane back to radial_tr.
__device__ __forceinline__ double radial_next(const double2 rr, double b0, double pm, double t, bool side, const TraceK& K,
                                              bool& outer) {
    const bool in_ok = (t < -b0) & (rr.x >= pm) & !side;
    const bool ch = !in_ok;
    const double r = ch ? rr.y : rr.x;
    const double disc = (r - pm) * (r + pm);
    const double sq = fast_sqrt_nan0(disc);
    const double sA = -b0 - sq, sB = sq - b0;
    const double dA = sA - t, dB = sB - t;
    const double tmin = (ch & !side) ? K.tol_same : K.tol;
    const bool ok = dA != dB;
    const bool vA = ok & (dA > tmin), vB = ok & (dB > tmin);
    outer = ch;
    return min_nonan(or_nan(vA, sA, K.nan_hi), or_nan(vB, sB, K.nan_hi));
}

// ---------------------------------------------- phi family, trace-relative (TREL) ---
// The half-plane through the z axis at phi_k meets the trace at s = num_k(p0) / den_k,
// num = x sin phi_k - y cos phi_k, den = n_y cos phi_k - n_x sin phi_k (ARTES.f90:3292-3350):
// linear in the trace parameter, so from the trace's start; family_eval1's rules for phi with
// the distances from the current point s - t (the half-plane the packet sits on, and the sp0
// quirk: the outer face vetoed when the inner one's root is >= 1e100, 3318, 3346).
__device__ __forceinline__ double phi_tr(const TraceTabs& T, double x0, double y0, double n0, double n1, double t, int tf,
                                         int cp, int pout, const TraceK& K, bool& outer) {
    const double2 sc0 = T.phsc[cp], sc1 = T.phsc[pout];
    const double den0 = n1 * sc0.y - n0 * sc0.x, num0 = x0 * sc0.x - y0 * sc0.y;
    const double den1 = n1 * sc1.y - n0 * sc1.x, num1 = x0 * sc1.x - y0 * sc1.y;
    const double sA = fast_div(num0, den0), sB = fast_div(num1, den1);
    const double dA = sA - t, dB = sB - t;
    const bool sameA = tf == cp + (2 << 16), sameB = tf == pout + (2 << 16);   // (phi face codes, face_code)
    const bool sp0_big = !sameA & (fabs(den0) > 0.0) & !(dA < K.huge);
    const bool vA = (fabs(den0) > K.tiny) & (dA > K.tol) & !sameA & (dA < K.huge);
    const bool vB = (fabs(den1) > K.tiny) & (dB > K.tol) & !(sameB | sp0_big) & (dB < K.huge);
    outer = vB & (!vA | (dB < dA));
    return min_nonan(or_nan(vA, sA), or_nan(vB, sB));
}

// Energy-transport diagnostics of a propagation segment (output:flow_global /
// output:flow_latitudinal).  add_flow_global (ARTES.f90:4992-5011): the direction's
// (r, theta, phi) components at the segment's end point, times segment length and
// Stokes I; add_flow (5013-5045): Stokes I through the cell's upper (lat 0) or lower
// (1) radial face, or its southern (2) or northern (3) theta face (lat -1: none).
__device__ __noinline__ void flow_segment(double* flow_g, double* flow_t, int cell, double x, double y, double z,
                                          double nx, double ny, double nz, double len, double w, int lat) {
    if (flow_g) {
        const double th = acos(z / sqrt(x * x + y * y + z * z));
        const double ph = atan2(y, x);
        const double st = sin(th), ct = cos(th), sp = sin(ph), cp = cos(ph);
        const double rd = st * cp * nx + st * sp * ny + ct * nz;
        const double td = ct * cp * nx + ct * sp * ny - st * nz;
        const double pd = -sp * nx + cp * ny;
        double* f = flow_g + 3 * (size_t)cell;
        atomicAdd(f + 0, rd * len * w);
        atomicAdd(f + 1, td * len * w);
        atomicAdd(f + 2, pd * len * w);
    }
    if (flow_t && lat >= 0) atomicAdd(flow_t + 4 * (size_t)cell + lat, w);
}

// -------------------------------------------------------------- k_trace ---
// A lane takes a slot from the trace list and runs its traces back to back as long as
// they chain inside the reference's packet loop: first optical depth -> propagation
// (forced first interaction, ARTES.f90:658-685) -> peel-off (scattering-loop head,
// 788-813) -> k_event.  Everything a chain needs is loaded once at refill and kept in
// registers (position, direction, RNG state, Stokes I); the slot is written back once
// when the chain ends, so no transition waits on memory.
//
// Per family the distance from the current position to its nearest face ahead is kept
// in a register (e0 radial, e1 theta, e2 phi; +inf: none) together with its side (bit f
// of `sides`: 0 inner, 1 outer face).  A step re-evaluates only the family crossed last
// (`pending`), picks the nearest of the three, moves there and subtracts the step from
// the other two.  The linear cell index is updated with the crossing, not recomputed.
//
// FLOW instantiations add the energy-transport diagnostics to propagation segments.
// NREP: steps per loop iteration (see the loop).
// GTAB: the face tables in global memory (G.ttab, k_fill_trace_tables) instead of LDS.
template <bool G3D, bool OBL, int WPE, bool FLOW = false, int NREP = 8, bool GTAB = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_trace(DevGrid G, DevRun R, Pool S, SubLists SL) {
    const Lists L = SL.l[sub_of_block()];
    extern __shared__ double s_tab[];
    const TraceTabs T = GTAB ? trace_tables_at(G, G.ttab) : stage_trace_tables(G, s_tab);
    const int n = *L.trace_in_n;
    const int split = *L.trace_in_split;   // [0, split): new packets' traces; then k_event's, stored backwards
    const int home = sub_block() & 7;
    __shared__ int s_q[2][QCAP * (BLOCK / 64)];
    const int wbase = QCAP * (threadIdx.x >> 6);
    WaveQueue q_event{&s_q[0][wbase], 0}, q_emit{&s_q[1][wbase], 0};
    // the wave's trace-list cursor lives in LDS between refills (a wave refills every ~10
    // iterations; kept in registers it occupied scalar registers that the step's lane masks
    // then had to be copied around, every iteration); only `exhausted` stays in a register
    // (3D grids without the flow diagnostics: the radial-only kernel keeps its 5th wave
    // per SIMD at <= 102 registers, the flow kernel has none to spare)
    const TraceK K = trace_consts<G3D && !FLOW>();
    __shared__ TraceCursor s_cur[BLOCK / 64];
    TraceCursor* const my_cur = &s_cur[threadIdx.x >> 6];
    bool exhausted;
    // the lookahead of the static deal (kernel_event.hpp, above load_chunk): the slot ids of
    // the wave's current and next static chunk, one per lane, and the prefetches' LDS sink
    [[maybe_unused]] int ck_cur = -1, ck_nxt = -1;
    __shared__ int s_pf_sink[64];
    [[maybe_unused]] const unsigned pf_sink = (unsigned)(uintptr_t)s_pf_sink;
    {
        const TraceCursor c0 = make_cursor(n, R.static_q64);
        if ((threadIdx.x & 63) == 0) *my_cur = c0;
        __builtin_amdgcn_wave_barrier();
        exhausted = c0.exhausted;
        if constexpr (LOOKAHEAD) {
            ck_cur = load_chunk(L.trace_in, c0.chunk, c0.nchunk, split, L.P);
            ck_nxt = load_chunk(L.trace_in, c0.chunk + c0.stride, c0.nchunk, split, L.P);

        }
    }
#ifdef ARTES_DEBUG_TIMING
    __shared__ unsigned long long s_tm[BLOCK / 64][20];
    unsigned long long* const my_tm = s_tm[threadIdx.x >> 6];
    if ((threadIdx.x & 63) < 20) my_tm[threadIdx.x & 63] = 0;
    __builtin_amdgcn_wave_barrier();
    auto tm_tick = [&]() -> unsigned long long {
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t = __builtin_readcyclecounter();
        __builtin_amdgcn_sched_barrier(0);
        return t;
    };
    auto tm_add = [&](int k, unsigned long long d) {   // by the wave's first active lane
        if ((int)(threadIdx.x & 63) == __builtin_ctzll(__ballot(true))) my_tm[k] += d;
    };
    TM_TICK(t_begin);
#endif
    const int fam_all = !G3D ? 1 : (G.nphi > 1 ? 7 : 3);
    const int nrt = G.nr * G.ntheta;        // linear-index stride of phi
    bool have = false;
#ifdef ARTES_DEBUG_LANES
    unsigned long long dbg_steps = 0, dbg_lanes = 0, dbg_refills = 0, dbg_tsteps = 0, dbg_tlanes = 0;
    unsigned long long dbg_anystop = 0, dbg_anyhit = 0, dbg_nstop = 0, dbg_nmove = 0, dbg_nretry = 0, dbg_nsetup = 0;
    unsigned long long dbg_firuns = 0, dbg_filanes = 0, dbg_reflanes = 0, dbg_hruns = 0, dbg_hlanes = 0;
    unsigned long long dbg_f12 = 0, dbg_anyf12 = 0;   // theta / phi evaluations: lanes, iterations with any
    unsigned long long dbg_f2 = 0, dbg_anyf2 = 0;     // the phi ones
    // per step of the unrolled iteration: lane-steps idle, parked, ended earlier, stepping, blocked
    unsigned long long dbg_rsteps = 0, dbg_ridle = 0, dbg_rpark = 0, dbg_rend = 0, dbg_rstep = 0, dbg_rblock = 0;
#endif
    // packet state (slot line 0) and trace state
    int slot = -1, mode = 0, pcell = 0, pface = 0, ncross = 0;
    double px = 0, py = 0, pz = 0, ttgt = 0, wI = 0;
    Rng rng{0, 0};
    int tcr = 0, tct = 0, tcp = 0, tf = -1, pending = 0, cell = 0;   // tf: face_code
    double tx = 0, ty = 0, tz = 0, nx = 0, ny = 0, nz = 0, tacc = 0, inz = 0, Axy = 0, Az = 0;
    // extinction and albedo weight of the current cell, loaded when the cell changes: the L2 round
    // trip overlaps the next iteration's face evaluation (one 16-byte load at a 32-bit byte
    // offset; ncell < 2^28, checked at grid creation)
    double kext = 0, gam = 0;
    auto load_cell = [&]() {
#ifdef ARTES_DEBUG
        if ((unsigned)cell >= (unsigned)G.ncell) {   // (ARTES_ERR_CELL: no out-of-range table read)
            log_err(R, ARTES_ERR_CELL);
            cell = 0;
        }
#endif
        const double2 kv = *(const double2*)((const char*)G.ka + ((unsigned)cell << 4));
        kext = kv.x;
        gam = kv.y;
    };
    // per family (radial, theta, phi) the distance to the nearest face ahead, and its
    // side (bit f of `sides`: 0 inner, 1 outer face)
    double e0 = INF, e1 = INF, e2 = INF;
    int sides = 0;
    // the radial family's side as the step direction of the shell index (+1: the outer sphere is
    // next, -1: the inner one), apart from `sides` (whose bit 0 the radial family then leaves
    // unused): the fused step adds it to the index as it is, and the evaluation writes it with one
    // select -- the bit's extraction, test and select and its insertion were five instructions
    int rdk = -1;
    // crossings: counted per packet (ncross, in the record) and added to the lane's total
    // once per chain, from the chain's start value nc0 (not per step)
    uint32_t c_cross = 0, c_peel = 0;
    int nc0 = 0;
    // backward propagation after the forced first interaction (see the FIRST-trace end).
    // During a first trace: the packet's crossings when it started.  During the backward
    // trace that may follow: 2 x crossings at its start + the first trace's steps + 1
    // (from which the forward walk's step count follows at the interaction).  0 otherwise.
    int kb = 0;
    int nlim = 0;   // the packet's crossing count at which the current trace is a runaway
    int parked = 0;   // 1: waiting for the batched forced first interaction (3: after a cell error)
    int pend = 0;     // the end mode of a chain whose list append waits for the wave's next refill
    int nt = 0;       // a new trace waits for the iteration's common set-up: NT_POS (the start cell) | NT_DIR
    // (3D grids; the radial-only kernel sets its cheap traces up where they start: the flag would
    // take it past 102 registers, its 5th wave per SIMD)
    constexpr bool SETUP_MERGED = G3D;

    // Lazy set-up (3D grids, one-face evaluation).  A new trace needs every family's
    // distance before its first step, one family per iteration, so two of every trace's
    // iterations used to move nothing.  Instead its three cache entries start as LOWER
    // BOUNDS of the distance to any face of the family, from the position alone: for the
    // spheres (r_out^2 - r^2) / (2 r_top) and (r^2 - r_in^2) / (2 r_top) (r +- r_k <= 2 r_top);
    // for a cone the distance to its two generator lines in the packet's meridional plane,
    // |rho cos th_k -+ z sin th_k| (the plane: |z|); for a phi half-plane the distance to
    // its plane, |x sin ph_k - y cos ph_k| -- each shrunk by 1e-9 relative and 1 um
    // absolute against rounding.  A family stays `pending` (bit f) while its entry is a
    // bound; a lane evaluates its pending families in order and steps as soon as the
    // nearest entry is an exact one beyond 1e-9 m: the reference's choice, since every
    // pending family's candidate lies at least as far as its bound (a candidate the rules
    // veto is farther still).  Bounds shrink by each step like the distances.  Elsewhere
    // (oblate grids, the two-face A/B build, the flow kernel, radial-only grids) the entries start at 0, so
    // every family is evaluated before the first step, as before.
    constexpr bool LAZY = G3D && !OBL && !TWOFACE && !FLOW;
    // Trace-relative radial family (radial_tr; the same kernels as the lazy set-up): the trace
    // keeps its start point (tx, ty, tz), its parameter tpar (the distance travelled) and the
    // family entries e0-e2 as trace parameters of their crossings, so a step moves tpar only;
    // the position p0 + tpar n is formed where it is needed (the theta / phi evaluation, the
    // interaction point, a trace's end).  b0 = p0.n and pm = |p0 x n| per trace.
    // (radial-only grids too: every crossing there is radial; ARTES_NO_TREL1D for A/B builds)
#ifdef ARTES_NO_TREL1D
    constexpr bool TREL = LAZY && TREL_ON;
#else
    constexpr bool TREL = (LAZY || (!G3D && !OBL && !TWOFACE && !FLOW)) && TREL_ON;
#endif
    double tpar = 0.0, b0 = 0.0, pm = 0.0;
#ifdef ARTES_NBF
    const double inv2rtop = LAZY ? 0.5 / sqrt(G.rf2[G.nr]) : 0.0;
#endif
    auto set_bounds = [&]() {
        if constexpr (LAZY) {
#ifdef ARTES_NBF
            const double r2 = fma(tx, tx, fma(ty, ty, tz * tz));
            const double br = min_nonan(T.fr[tcr + 1].off - r2, r2 - T.fr[tcr].off) * inv2rtop;
#else
            // (the radial family is the lowest pending bit, so a new trace evaluates it in its
            // first iteration, before any step reads e0: its bound would never be read)
            const double br = 0.0;
#endif
            const double rho = fast_sqrt(fma(tx, tx, ty * ty));
            const double2 c0 = T.tcs[tct], c1 = T.tcs[tct + 1];
            const double bt = min_nonan(min_nonan(fabs(fma(rho, c0.x, -tz * c0.y)), fabs(fma(rho, c0.x, tz * c0.y))),
                                        min_nonan(fabs(fma(rho, c1.x, -tz * c1.y)), fabs(fma(rho, c1.x, tz * c1.y))));
            double bp = K.inf;
            if (G.nphi > 1) {
                const double2 s0 = T.phsc[tcp], s1 = T.phsc[tcp + 1 == G.nphi ? 0 : tcp + 1];
                bp = min_nonan(fabs(fma(tx, s0.x, -ty * s0.y)), fabs(fma(tx, s1.x, -ty * s1.y)));
            }
            e0 = fma(br, 1.0 - 1.e-9, -1.e-6);
            e1 = fma(bt, 1.0 - 1.e-9, -1.e-6);
            e2 = fma(bp, 1.0 - 1.e-9, -1.e-6);
        } else {
            e0 = 0.0; e1 = 0.0; e2 = 0.0;
        }
    };
    // the trace-relative constants of a trace starting at (tx, ty, tz) along n
    auto set_trel = [&]() {
        if constexpr (TREL) {
            tpar = 0.0;
            b0 = fma(tx, nx, fma(ty, ny, tz * nz));
            const double cx = fma(ty, nz, -tz * ny), cy = fma(tz, nx, -tx * nz), cz = fma(tx, ny, -ty * nx);
            pm = fast_sqrt(fma(cx, cx, fma(cy, cy, cz * cz)));
        }
    };
    // a new direction with its per-trace constants, and a fresh family cache
    const double ax2 = OBL ? G.ax2 : 1.0, by2 = OBL ? G.by2 : 1.0, cz2 = OBL ? G.cz2 : 1.0;
    // (TREL: Axy, Az and 1/n_z only feed the rare theta / phi evaluation, which forms them
    // itself: no registers across the loop)
    auto set_direction = [&](double d0, double d1, double d2) {
        nx = d0; ny = d1; nz = d2;
        if constexpr (!TREL) {
            Axy = dir_axy(ax2, by2, nx, ny);
            Az = cz2 * nz * nz;
        }
        tacc = 0.0;
        nlim = ncross + (1 << 22);
        pending = fam_all;
        sides = 0;
        rdk = -1;
        set_bounds();
        if constexpr (G3D && !TREL) inz = fast_rcp(nz);
        set_trel();
    };
    // a trace starts at the packet position with zero optical depth
    auto start_position = [&]() {
        tx = px; ty = py; tz = pz;
        unpack_cell(pcell, tcr, tct, tcp);
        {
            int ft, fi;
            unpack_face(pface, ft, fi);
            tf = face_code(ft, fi);
        }
#ifdef ARTES_DEBUG
        if (tcr >= G.nr || tct >= G.ntheta || tcp >= G.nphi) {   // (ARTES_ERR_CELL: the run fails; no out-of-range read)
            log_err(R, ARTES_ERR_CELL);
            tcr = min(tcr, G.nr - 1); tct = min(tct, G.ntheta - 1); tcp = min(tcp, G.nphi - 1);
        }
#endif
        cell = tcr + (int)__umul24((unsigned)G.nr, (unsigned)tct) + (int)__umul24((unsigned)nrt, (unsigned)tcp);
        load_cell();
    };

    // The forced first interaction at the end of a first trace (ARTES.f90:658-685): one
    // exp and one log, ~140 VALU instructions, needed by about one lane in three
    // wave-steps.  The lane parks instead and the wave runs the block for all parked lanes
    // together once R.batch of them wait (or few lanes are still stepping).
    auto first_interaction = [&](bool err) {
        // one exp and one log for every case: e = 1 outside [1e-6, 50)
        const double tau_first = tacc;
        const double xi = rng.uni();
        const bool mid = tau_first >= 1.e-6 && tau_first < 50.0;
        const double e = mid ? 1.0 - exp(-tau_first) : 1.0;
        const double tau = -log(1.0 - xi * e);
        if (mid) wI *= e;
        mode = S_PROP;
        // The propagation that follows walks the first trace's chord again, from its start
        // to optical depth tau (ARTES.f90:689-720).  When the interaction lies in the
        // chord's far half it is reached in fewer cells from the far end: walk back from
        // where the first trace stopped (tx, tf, cell: set when the lane parked) to
        // optical depth tau_first - tau.  Same cells in reverse, so the same interaction
        // point up to rounding; crossing counts are kept as the forward walk's (kb).  Not
        // with the flow diagnostics (segment order).
        bool back = false;
        if constexpr (!FLOW) back = R.backward && mid && !err && tau_first - tau < tau;
        kb = back ? 2 * ncross + (ncross - kb) + 1 : 0;
        // (one set_direction for both walks, on selected operands: the two inlined copies ran
        // as a divergent pair, ~65 VALU instructions more per block)
        // (3D grids: the new trace's set-up waits for the iteration's common set-up block, below)
        ttgt = back ? fmax(tau_first - tau, 0.0) : tau;   // (tau rounds to <= tau_first + 1 ulp)
        if (back) { nx = -nx; ny = -ny; nz = -nz; }
        if constexpr (SETUP_MERGED) {
            nt = back ? NT_DIR : NT_POS | NT_DIR;
        } else {
            if (!back) start_position();
            set_direction(nx, ny, nz);
        }
    };

    // The interaction at the end of a propagation (ARTES.f90:705-720), then the
    // scattering-loop head (788-813): roulette, albedo weight, minimum weight, and the
    // peel-off trace's start.  About 85 VALU instructions for the one or two lanes of a
    // wave-step that reach their interaction point; those lanes park (4) instead and the
    // wave runs the block for R.hbatch of them together.  Returns the slot's end mode
    // (absorbed) or 0 (the peel-off trace goes on in this lane).
    auto interaction = [&]() -> int {
        const double s = fast_div(ttgt - tacc, kext) + (TREL ? tpar : 0.0);   // (TREL: from the trace's start)
        px = tx + s * nx; py = ty + s * ny; pz = tz + s * nz;
#ifdef ARTES_DEBUG_GEOM
        {   // diagnostic build: is the interaction point in the cell's radial shell?
            const double S2 = ax2 * px * px + by2 * py * py + cz2 * pz * pz;
            if (S2 < G.rf2[tcr] * (1 - 1e-9) || S2 > G.rf2[tcr + 1] * (1 + 1e-9)) {
                if (atomicAdd(&R.err[ARTES_ERR_GEOM], 1ULL) < 6)
                    printf("[geom] hit outside shell: t %.17g %.17g %.17g n %.17g %.17g %.17g cell %d %d %d face %d %d e %.17g %.17g %.17g sides %x s %.17g steps left %d mode %d S2/rf2 %.17g %.17g\n",
                           tx, ty, tz, nx, ny, nz, tcr, tct, tcp, face_code_type(tf), face_code_index(tf), e0, e1, e2, sides, s, nlim - ncross, mode,
                           S2 / G.rf2[tcr], S2 / G.rf2[tcr + 1]);
            }
        }
#endif
        pcell = pack_cell(tcr, tct, tcp);
        // an interaction point lies on no face; until k_event starts the next trace the face
        // field carries the cell's scattering-matrix id instead, so k_event needs no dependent
        // read of the per-cell id table (k_event resets it to 0).  The load's result is only
        // stored at the chain's end.
        pface = G.nmat > 1 ? G.matid[cell] : 0;
        if (kb) {   // a backward trace: count the steps the forward one takes
            ncross = kb - ncross;
            kb = 0;
        }
        if constexpr (FLOW) flow_segment(R.flow_g, R.flow_t, cell, px, py, pz, nx, ny, nz, s, wI, -1);   // (715, 874)
        const double xi = rng.uni();   // a killed packet's RNG state is not used again
        bool kill = !R.photon_scattering || xi < R.fstop;
        wI *= gam;   // albedo / (1 - fstop) where 0 < albedo < 1, else 1 (ARTES.f90:801-805; the table, transport.hip)
        __builtin_amdgcn_sched_barrier(0);   // (a scheduling boundary, as the old branch was: 5 registers fewer)
        kill = kill || wI <= R.pmin;
        if (kill) return S_END_ABS;
        // peel-off trace (ARTES.f90:4722-4761) from the interaction point: same cell (kext,
        // gam stay), no face
        c_peel++;
        mode = S_PEEL;
        tx = px; ty = py; tz = pz;
        tf = -1;
        nx = R.det0; ny = R.det1; nz = R.det2;
        if constexpr (SETUP_MERGED) nt = NT_DIR;   // (the set-up: the iteration's common block, below)
        else set_direction(nx, ny, nz);
        return 0;
    };

    // A chain that ends writes its record back at once; its slot is appended to the event or
    // emit list by `append` (call with the whole wave: the appends are wave-aggregated) at
    // the end of the iteration, or with R.late_append at the wave's next refill (and after the
    // loop): one append block for the ~16 lanes of a refill instead of two in every iteration.
    // (Deferring the record stores too kept the ended packets' state live across iterations:
    // 16 spilled registers.)
    auto append = [&]() {
        q_event.push(pend && to_event_list(pend), slot);
        q_emit.push(pend && !to_event_list(pend), emit_entry(slot, pend));
        pend = 0;
    };

    // The evaluated family's entry is exact now: clear ITS pending bit (fam is always a pending
    // family, so the xor clears it; two instructions, as `pending & (pending - 1)`).  (The
    // round-2 "nearest bound first" variant evaluated a family other than the lowest pending one
    // but kept `pending &= pending - 1`, which clears the LOWEST bit: that family's bound was
    // then taken for an exact distance, the lane stepped onto it as onto a face, and next_cell
    // walked the cell indices out of range -- the illegal access of that round, DESIGN.md §4;
    // ARTES_DEBUG counts such a clear as ARTES_ERR_PENDING.  The trace-relative kernels now
    // evaluate the nearest pending bound first, with this clear.)
    auto clear_pending = [&](int fam, bool retry) __attribute__((always_inline)) {
#ifdef ARTES_DEBUG
        const int pending_before = pending;
#endif
#ifdef ARTES_OLD_CLEAR
        if (!retry) pending &= pending - 1;   // (development build: the round-2 clear)
#else
        if (!retry) pending ^= 1 << fam;
#endif
#ifdef ARTES_DEBUG
        if (!retry && (pending_before & ~pending) != (1 << fam)) log_err(R, ARTES_ERR_PENDING);
#endif
    };

    // watchdog: a wave runs ~1e4 iterations per launch at the largest pool; a schedule bug
    // must not leave waves spinning on the device (the run then fails with error 57)
    unsigned int iters_left = 1u << 24;
    for (;;) {
        if (--iters_left == 0) {
            if ((threadIdx.x & 63) == 0) atomicAdd(&R.err[ARTES_ERR_WATCHDOG], 1ULL);
            break;
        }
        int end = 0;   // 0: continue, else the slot's new mode
        TM_TICK(t0);
        {
            const unsigned long long pk = __ballot(parked != 0);
            if (pk) {
                const int stepping = __popcll(__ballot(have && parked == 0));
                // (stepping == 0: every busy lane is parked, and the idle ones may be too few to
                // refill -- waiting for more would never end)
                const bool force = stepping < R.batch_min || stepping == 0 || exhausted;
                const unsigned long long pf = __ballot(parked & 1), ph = pk & ~pf;
                if (pf && (__popcll(pf) >= R.batch || force)) {
#ifdef ARTES_DEBUG_LANES
                    dbg_firuns++;
                    dbg_filanes += __popcll(pf);
#endif
                    TM_TICK(tf0);
                    if (parked & 1) {
                        first_interaction(parked & 2);
                        parked = 0;
                    }
                    TM_TICK(tf1);
                    TM_ADD(13, tf1 - tf0);
                }
                if (ph && (__popcll(ph) >= R.hbatch || force)) {
#ifdef ARTES_DEBUG_LANES
                    dbg_hruns++;
                    dbg_hlanes += __popcll(ph);
#endif
                    TM_TICK(th0);
                    if (parked == 4) {
                        end = interaction();
                        parked = 0;
                    }
                    TM_TICK(th1);
                    TM_ADD(14, th1 - th0);
                }
            }
        }
        TM_TICK(t1);
        TM_ADD(0, t1 - t0);
        // ---------------------------------------------------------------- refill
        if (!exhausted) {
            const unsigned long long idle = __ballot(!have);
            if (__popcll(idle) >= R.refill || idle == __ballot(true)) {
                append();
                TM_TICK(tr_a);
                TM_ADD(8, tr_a - t1);
                TraceCursor cur = load_cursor(my_cur);
                int my;
                if constexpr (LOOKAHEAD) {
                    int sl;
                    my = wave_take<true>(cur, L.grab, home, !have, R.dgrab, &sl, &ck_cur, &ck_nxt, &L, split, S.s, pf_sink);
                    if (!have && my >= 0) slot = sl != -2 ? sl : L.trace_in[list_pos(my, split, L.P)];
                } else {
#ifdef ARTES_DEBUG_TIMING
                    int n_atom = 0;
                    my = wave_take(cur, L.grab, home, !have, R.dgrab, nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0, &n_atom);
#else
                    my = wave_take(cur, L.grab, home, !have, R.dgrab);
#endif
                    TM_TICK(tr_b);
                    TM_ADD(9, tr_b - tr_a);
#ifdef ARTES_DEBUG_TIMING
                    // takes that issued dynamic grabs (atomics): their cycles, their count; all takes; grabs
                    if (n_atom) { TM_ADD(16, tr_b - tr_a); TM_ADD(17, 1); }
                    TM_ADD(18, 1);
                    TM_ADD(19, n_atom);
#endif
                    if (!have && my >= 0) slot = L.trace_in[list_pos(my, split, L.P)];
#ifdef ARTES_DEBUG_TIMING
                    asm volatile("" ::"v"(slot));   // (the list entry's wait inside this region)
                    my_tm[15] = tm_tick() - tr_b;   // (lane-0 scratch: added below)
#endif
                }
                TM_TICK(tr_c);
#ifdef ARTES_DEBUG_TIMING
                __builtin_amdgcn_wave_barrier();
                if (!LOOKAHEAD) TM_ADD(10, my_tm[15]);
#endif
                if ((threadIdx.x & 63) == 0) *my_cur = cur;
                __builtin_amdgcn_wave_barrier();
                exhausted = cur.exhausted;
#ifdef ARTES_DEBUG_LANES
                dbg_refills++;
#endif
#ifdef ARTES_DEBUG
                if (!have && my >= 0) {
                    const int pos = my < split ? my : L.P - 1 - (my - split);
                    const int m = (slot >= 0 && slot < S.P) ? S.s[slot].mode : S_FIRST;
                    dbg_claim(R, L, (my < n && pos >= 0 && pos < L.P) ? slot : -2, S.P, 0, m == S_FIRST || m == S_PROP || is_peel_trace(m));
                }
#endif
#ifdef ARTES_DEBUG_LANES
                dbg_reflanes += __popcll(__ballot(!have && my >= 0 && slot >= 0));
#endif
#ifdef ARTES_DEBUG_TIMING
                unsigned long long tr_d = tm_tick();
                bool did = false;
#endif
                if (!have && my >= 0 && slot >= 0) {   // -1: a hole left by a dropped or retired packet
                    const Slot* rec = S.s + slot;
                    mode = rec->mode;
                    px = rec->px; py = rec->py; pz = rec->pz;
                    const double ldx = rec->dx, ldy = rec->dy, ldz = rec->dz;
                    ttgt = rec->ttgt;
                    rng.s0 = rec->r0; rng.s1 = rec->r1;
                    pcell = rec->pcell; pface = rec->pface;
                    ncross = rec->ncross;
                    nc0 = ncross;
                    wI = rec->wI;
#ifdef ARTES_DEBUG_TIMING
                    asm volatile("" ::"v"(px), "v"(wI), "v"(ncross), "v"(ldz));   // (the record's wait before the set-up)
                    tr_d = tm_tick();
                    did = true;
#endif
                    const bool peel = is_peel_trace(mode);
                    nx = peel ? R.det0 : ldx; ny = peel ? R.det1 : ldy; nz = peel ? R.det2 : ldz;
                    if constexpr (SETUP_MERGED) {
                        nt = NT_POS | NT_DIR;   // (the set-up: the common block below)
                    } else {
                        start_position();
                        set_direction(nx, ny, nz);
                    }
                    have = true;
                    kb = (mode == S_FIRST) ? ncross : 0;
                }
#ifdef ARTES_DEBUG_TIMING
                {   // record loads / set-up split at the first refilling lane's clock
                    TM_TICK(tr_e);
                    const unsigned long long rb = __ballot(did);
                    if (rb) {
                        const int fl = __builtin_ctzll(rb);
                        const unsigned long long td = ((unsigned long long)(unsigned)__shfl((int)(tr_d >> 32), fl) << 32) |
                                                      (unsigned)__shfl((int)tr_d, fl);
                        TM_ADD(11, td - tr_c);
                        TM_ADD(12, tr_e - td);
                    } else {
                        TM_ADD(11, tr_e - tr_c);
                    }
                }
#endif
            }
        }
        // The new traces of this iteration -- the forced first interactions' propagations, the
        // interactions' peel-offs and the refilled slots' traces -- set up together: the start
        // cell (unless a backward walk starts where the first trace stopped), the direction's
        // constants, the lazy bounds and the trace-relative constants run once per iteration for
        // all of them, instead of once in each of the three blocks
        if (SETUP_MERGED && __ballot(nt != 0)) {
            TM_TICK(ts0);
            if (nt & NT_POS) start_position();
            if (nt) set_direction(nx, ny, nz);
            nt = 0;
            TM_TICK(ts1);
            TM_ADD(12, ts1 - ts0);
        }
        TM_TICK(t2);
        TM_ADD(1, t2 - t1);
        if (!__any(have) && exhausted) break;   // (all lanes idle otherwise: every grab was a hole)
#ifdef ARTES_DEBUG_LANES
        dbg_steps++;
        dbg_lanes += __popcll(__ballot(have));
        if (exhausted) { dbg_tsteps++; dbg_tlanes += __popcll(__ballot(have)); }
#endif
#ifdef ARTES_DEBUG_LANES
        bool dbg_s = false, dbg_h = false, dbg_m = false, dbg_r = false, dbg_u = false;
#endif
        // The evaluation and the step, NREP times per iteration (unrolled): the iteration's
        // wave-level blocks -- parked-lane ballots and blocks, refill check and refill,
        // chain-end stores, queue flushes, loop head -- run once per NREP steps.  A lane that
        // ends or parks sits out the rest of the iteration ("Several steps per
        // iteration").  (A compile-time count: a runtime one, a scalar compare per copy, cost
        // ray3d 3 %.)
        // Trace-relative kernels: NREP steps in the radial form (a sphere beyond 1e-9 m: ~99.9 % of
        // the crossings on the bench grid, 99.6 % on the cloudy one), then one generic step for
        // every family and the reference's two-pass choice.  (The generic slot taking the fused
        // radial step for its radial lanes too measured slower: ray3d k_trace +1.7 %, hg +1.6 %,
        // profiles/r06/ab/trace_mixed_generic_slot_ab.txt.)  A lane whose next crossing is a
        // theta / phi face, or lies within 1e-9 m, waits for that last step of the iteration: the
        // radial form is then a straight sequence of instructions with no per-lane choice of the
        // crossed family's index, no phi wrap and no index selects, and no join of two step forms
        // (whose register copies cost more than the selects they saved).
        constexpr int NSLOT = TREL ? NREP + 1 : NREP;
#pragma unroll
        for (int rep = 0; rep < NSLOT; rep++) {
        const bool generic_slot = !TREL || rep == NREP;   // (a constant in every unrolled copy)
        TM_TICK(t_rep);   // (timing build: the evaluation is timed from each step's start)
#ifdef ARTES_DEBUG_LANES
        {   // per step: lanes idle, parked, ended in an earlier step of the iteration
            dbg_rsteps++;
            dbg_ridle += __popcll(__ballot(!have));
            dbg_rpark += __popcll(__ballot(have && parked));
            dbg_rend += __popcll(__ballot(have && !parked && end));
        }
#endif
        if (have && !parked && !end) {
            const double k = kext;
            // the nearest entry (TREL: a trace parameter) and its family; its distance from the
            // current point; whether the lane steps
            double best_abs, best;
            int w;
            bool fast, do_step;
            bool rstep = false;   // (radial-form slots: the fused radial step)
            double bestr = 0.0;
            if constexpr (TREL) {
                // A. The radial family, whenever its entry is not exact (pending bit 0): the last
                // step crossed a sphere (99.9 % of all crossings on the bench grid), a trace starts,
                // or the chosen sphere had no crossing (`alt`: the other one).  No per-lane choice
                // of the family to evaluate: every lane that evaluates at all evaluates this one.
                if (pending & 1) {
                    const bool alt = (sides >> 4) & 1;
                    bool outer;
                    const double dm = radial_tr(T, b0, pm, tpar, tf, tcr, alt, K, outer);
                    const bool retry = !alt & !(dm < K.inf);
                    // (the other face is still to come: the entry is the current trace parameter,
                    // the nearest one, and the bit stays pending)
                    e0 = retry ? tpar : dm;
                    sides = (sides & ~0x10) | (retry ? 16 : 0);
                    rdk = outer ? 1 : -1;
                    clear_pending(0, retry);
#ifdef ARTES_DEBUG_LANES
                    dbg_r = retry; dbg_u = true;
#endif
                }
                // A'. Radial-form slots: the lane steps onto its sphere when the radial entry is
                // exact, the nearest one (ties to the radial family; NaN theta / phi entries are no
                // candidates) and beyond 1e-9 m -- B's choice with w = 0 and a fast step (a radial
                // entry is finite or NaN, never +inf).  B and C below run only when some lane of
                // the wave does neither this nor A again but has a theta / phi bound pending.
                if (!generic_slot) {
                    bestr = e0 - tpar;
                    rstep = !(pending & 1) & (bestr > K.step_min);
                    if constexpr (G3D) rstep = rstep & !(e0 > min_nonan(e1, e2));
                }
                do_step = false;
                best_abs = e0; best = bestr; w = 0; fast = rstep;
                if (generic_slot || (G3D && __ballot(!rstep & (pending != 0) & !(pending & 1)))) {
                // B. The choice: the nearest of the three entries.  A lane steps unless a pending
                // family blocks it -- its bound is the nearest entry, or some family is pending and
                // nothing lies beyond 1e-9 m -- (the reference's choice whenever it steps: a pending
                // family's candidate lies at least as far as its bound, DESIGN.md §4 "Lazy set-up")
                best_abs = e0;
                w = 0;
                if constexpr (G3D) {
                    best_abs = min_nonan(min_nonan(e0, e1), e2);
                    w = e0 == best_abs ? 0 : (e1 == best_abs ? 1 : 2);
                }
                best = best_abs - tpar;
                fast = best > K.step_min && best < K.inf;
                const bool blocked = ((pending >> w) & 1) | (!fast & (pending != 0));
                // C. Theta / phi (3D grids): the blocking family when it is one of them (a lane whose
                // radial entry is still pending runs A again in its next step) -- the nearest pending
                // bound first (w), or the lowest pending family when nothing lies beyond 1e-9 m.
                // Theta evaluations (the quadratic from the current point) are batched in the
                // 4-step kernel (coarse grids: short traces, many set-up evaluations): a lane that
                // needs one waits until R.gbatch lanes of the wave do, or few lanes still step.
                // The 8-step kernel evaluates at once (waiting measured 3.5 % slower on ray3d), with
                // no ballots or counts (k_trace -2 %; profiles/r05/ab/trace_theta_unbatched_*).
                if constexpr (G3D) {
                    constexpr bool TBATCH = NREP < 8;
                    const bool tp = blocked && !(pending & 1);
                    [[maybe_unused]] const unsigned long long act = TBATCH ? __ballot(true) : 0;
                    if (!TBATCH || __ballot(tp)) {   // (a wave-uniform test first: ~10 % of the steps need this)
                    const int fam = fast ? w : __builtin_ctz(pending & 6);
                    // (both ballots outside any short-circuit: under `||` the second one would count
                    // only the lanes that reach it)
                    [[maybe_unused]] const unsigned long long gm = TBATCH ? __ballot(tp && fam == 1) : 0;
#ifdef ARTES_DEBUG_LANES
                    const unsigned long long pm2 = __ballot(tp && fam == 2);
#endif
                    {
                        bool run = TBATCH ? (tp && fam == 2) : tp;
                        if (TBATCH && gm) {
                            const int ng = __popcll(gm);
                            const bool go = ng >= R.gbatch || __popcll(act) - ng < R.batch_min || exhausted;
                            run = run || (tp && fam == 1 && go);
                        }
                        if (run) {
                            const int pout = (tcp + 1 == G.nphi) ? 0 : tcp + 1;
                            const bool alt = (sides >> (4 + fam)) & 1;
                            bool outer;
                            double dm;
                            if (fam == 2) {
                                dm = phi_tr(T, tx, ty, nx, ny, tpar, tf, tcp, pout, K, outer);
                            } else {   // theta (~0.1-0.4 % of crossings): from the current point
                                TM_TICK(ta);
                                const double qx = fma(tpar, nx, tx), qy = fma(tpar, ny, ty), qz = fma(tpar, nz, tz);
                                dm = tpar + family_eval1<G3D, OBL, true>(G, T, fam, qx, qy, qz, nx, ny, nz, dir_axy(ax2, by2, nx, ny),
                                                                         cz2 * nz * nz, tf, tcr, tct, tcp, pout, -qz * fast_rcp(nz),
                                                                         alt, K, outer);
                                TM_TICK(tb);
                                TM_ADD(5, tb - ta);
                            }
                            const bool retry = (fam == 1) & !alt & !(dm < K.inf);
                            dm = retry ? tpar : dm;
                            e1 = fam == 1 ? dm : e1;
                            e2 = fam == 2 ? dm : e2;
                            sides = (sides & ~(0x11 << fam)) | (((outer ? 1 : 0) | (retry ? 16 : 0)) << fam);
                            clear_pending(fam, retry);
#ifdef ARTES_DEBUG_LANES
                            dbg_r = retry; dbg_u = true;
#endif
                        }
#ifdef ARTES_DEBUG_LANES
                        dbg_f12 += __popcll(gm | pm2);
                        dbg_anyf12 += 1;
                        dbg_f2 += __popcll(pm2);
                        dbg_anyf2 += pm2 != 0;
#endif
                    }
                    }   // any tp
                }
                // D. The step below (a lane that evaluated theta / phi above steps in its next one)
                do_step = !blocked;
                }   // B, C
                TM_TICK(tev);
                TM_ADD(2, tev - t_rep);
            } else {
                // ------------------------------------------- evaluate one face family
    #ifdef ARTES_NBF
                // development variant: the pending family with the nearest bound first
                int fam = 0;
                if constexpr (G3D) {
                    const double b0 = (pending & 1) ? e0 : INF, b1 = (pending & 2) ? e1 : INF, b2 = (pending & 4) ? e2 : INF;
                    fam = (b0 <= b1 && b0 <= b2) ? 0 : (b1 <= b2 ? 1 : 2);
                    fam = ((pending >> fam) & 1) ? fam : __builtin_ctz(pending);
                }
    #else
                const int fam = G3D ? __builtin_ctz(pending) : 0;
    #endif
                const int pout = G3D ? ((tcp + 1 == G.nphi) ? 0 : tcp + 1) : 0;
                bool outer;
                // the face the family can cross next; the other one if that has no crossing
                // (`alt`, bit 4 + fam of `sides`: evaluated in this lane's next iteration).  Both
                // faces on an oblate grid: there the star's packets start inside the atmosphere's
                // outer surface (the reference emits them on the unscaled sphere), a position its
                // cell does not contain, where the nearest crossing is not the one the direction
                // points to
                double dm;
                bool retry = false;
                if constexpr (OBL || TWOFACE) {
                    dm = family_eval<G3D, OBL>(G, T, fam, tx, ty, tz, nx, ny, nz, Axy, Az, tf, tcr, tct, tcp, pout, -tz * inz, outer);
                } else {
                    const bool alt = (sides >> (4 + fam)) & 1;
                    dm = family_eval1<G3D, OBL>(G, T, fam, tx, ty, tz, nx, ny, nz, Axy, Az, tf, tcr, tct, tcp, pout, -tz * inz, alt, K, outer);
                    retry = (fam != 2) & !alt & !(dm < K.inf);
                }
                // (the other face is still to come: no bound.  Only the high word is cleared: the
                // entry is then 0 or a positive denormal, below any step, so the family stays the
                // nearest pending one exactly as with 0)
                if constexpr (LAZY) dm = __hiloint2double(retry ? 0 : __double2hiint(dm), __double2loint(dm));
                if constexpr (G3D) {
                    e0 = fam == 0 ? dm : e0;
                    e1 = fam == 1 ? dm : e1;
                    e2 = fam == 2 ? dm : e2;
                    sides = (sides & ~(0x11 << fam)) | (((outer ? 1 : 0) | (retry ? 16 : 0)) << fam);
                    rdk = fam == 0 ? (outer ? 1 : -1) : rdk;
                } else {
                    e0 = dm;
                    sides = (outer ? 1 : 0) | ((retry ? 1 : 0) << 4);
                    rdk = outer ? 1 : -1;
                }
                // the evaluated family's entry is exact now: clear ITS bit (see clear_pending)
                clear_pending(fam, retry);
    #ifdef ARTES_DEBUG_LANES
                dbg_r = retry; dbg_u = true;   // (evaluated; lanes that also step are subtracted below)
    #endif
                TM_TICK(tev);
                TM_ADD(2, tev - t_rep);
                // ---------------------------------------------------- trace step
                // nearest face, 'large' then 'small' solutions (ARTES.f90:3358-3418)
                // The nearest distance of the three is the reference's choice whenever it
                // exceeds 1e-9 m (then all of them do); the two-pass rule runs only when it
                // does not (a crossing at a corner of two families) or nothing is ahead.
                // (NaN: no crossing; ties go to the lower family, as the reference's order.)
                // With pending families (bounds), only an exact nearest entry beyond 1e-9 m steps.
                // (TREL: the entries are trace parameters; best_abs the nearest one, best its distance)
                best_abs = e0;
                w = 0;
                if constexpr (G3D) {
                    best_abs = min_nonan(min_nonan(e0, e1), e2);
                    w = e0 == best_abs ? 0 : (e1 == best_abs ? 1 : 2);
                }
                best = best_abs;
                fast = best > K.step_min && best < K.inf;
                do_step = pending == 0 || (LAZY && fast && !((pending >> w) & 1));
            }
            // ---------------------------------------------------- the step
            // From the nearest entry best_abs of family w: the reference's two-pass choice when
            // that is not beyond 1e-9 m (ARTES.f90:3358-3418), next_cell (2671-2798), the
            // optical-depth sum and the trace ends (625-778, 848-941, 4739-4761)
#ifdef ARTES_DEBUG_LANES
            dbg_rstep += __popcll(__ballot(generic_slot ? do_step : rstep));
            dbg_rblock += __popcll(__ballot(!(generic_slot ? do_step : rstep)));
#endif
            if (!generic_slot) {
                if (rstep) {
                    // The fused radial step (trace-relative kernels, see NSLOT): the generic step
                    // below with w = 0 and a fast choice, the same results, and then at once the
                    // radial family of the new shell (radial_next: radial_tr's result for the packet
                    // on the sphere it just crossed), so the lane's next slot needs no evaluation.
                    // The new shell's radii are read before the trace-end tests (rr[kn] for
                    // kn = -1 .. nr: padded, used only when the packet stays in the grid).
                    const int dk = rdk;
                    const bool side = dk > 0;
                    // (kn out of the compiler's sight: the new shell's index for the radii read and the
                    // face, while tcr moves in place below -- as one value the two branches' tcr met in
                    // two copies at the join)
                    int kn;
                    asm("v_add_u32 %0, %1, %2" : "=v"(kn) : "v"(tcr), "v"(dk));
                    const double2 rrn = T.rr[kn];
                    const int nfi = side ? kn : tcr;
                    // (a runaway trace -- 2^22 crossings -- is stopped at the end of the iteration, below)
                    const bool exit = side & (nfi == G.nr);
                    const bool surf = nfi == G.cell_depth;
                    bool err = (tf == G.cell_depth) & surf;
    #ifdef ARTES_DEBUG
                    if (!err && !exit && !surf && (kn < 0 || kn >= G.nr)) {   // (ARTES_ERR_CELL, as below)
                        log_err(R, ARTES_ERR_CELL);
                        err = true;
                    }
    #endif
                    ncross++;
                    const double tau_cell = bestr * k;
                    const bool prop = (mode == S_PROP);
                    const bool hit = prop && tacc + tau_cell > ttgt;
                    const bool stop = err || exit || surf || hit;
    #ifdef ARTES_DEBUG_LANES
                    dbg_s = stop; dbg_h = prop && hit && !err; dbg_m = !stop; dbg_u = false;
    #endif
                    const bool hitpark = prop & hit & !err;
                    if (!hitpark) {
                        tacc += tau_cell;
                        tpar = e0;
                    }
                    // (the face also for a lane whose interaction lies in this cell: interaction()
                    // resets it before the peel-off, and an absorbed packet's face is dead)
                    tf = nfi;
                    if (!stop) {
                        cell += dk;
                        tcr += dk;
                        load_cell();
                        bool outer;
                        const double dm = radial_next(rrn, b0, pm, tpar, side, K, outer);
                        e0 = dm;
                        rdk = outer ? 1 : -1;
                        pending |= (dm < K.inf) ? 0 : 1;   // (NaN: radial_tr in the next slot, alt)
                    } else {
                        // (the end's reasons follow from the state at the end of the iteration: PK_RAD)
                        parked = hitpark ? 4 : (err ? PK_RAD_ERR : PK_RAD_END);
                    }
                }   // rstep
            } else if (do_step) {
                {
                    if (!fast) {   // rare (every family exact here)
                        const double r0 = TREL ? e0 - tpar : e0, r1 = TREL ? e1 - tpar : e1, r2 = TREL ? e2 - tpar : e2;
                        const double t0 = or_nan(r0 > 1.e-9, r0);
                        best = t0;
                        w = 0;
                        if constexpr (G3D) {
                            const double t1 = or_nan(r1 > 1.e-9, r1), t2 = or_nan(r2 > 1.e-9, r2);
                            best = min_nonan(min_nonan(t0, t1), t2);
                            w = t0 == best ? 0 : (t1 == best ? 1 : 2);
                        }
                        if (!(best < INF)) {   // nothing beyond 1e-9 m
                            best = r0 > 1.e-12 ? r0 : INF;
                            w = 0;
                            if constexpr (G3D) {
                                if (r1 > 1.e-12 && r1 < best) { best = r1; w = 1; }
                                if (r2 > 1.e-12 && r2 < best) { best = r2; w = 2; }
                            }
                        }
                        best_abs = w == 0 ? e0 : (w == 1 ? e1 : e2);
                    }
                    // next_cell (ARTES.f90:2671-2798): the crossed family's index moves by one
                    // (phi wraps); the face index is the old one (inner face) or the new one
                    // (outer face) for every family
                    const bool side = w == 0 ? rdk > 0 : ((sides >> w) & 1);
                    const int kf = !G3D ? tcr : (w == 0 ? tcr : (w == 1 ? tct : tcp));
                    int kn = kf + (side ? 1 : -1);
                    if constexpr (G3D) {   // (branch-free: a divergent branch costs more scalar work)
                        const int wrapped = kn < 0 ? G.nphi - 1 : (kn == G.nphi ? 0 : kn);
                        kn = w == 2 ? wrapped : kn;
                    }
                    const int nfi = side ? kn : kf;
                    // a trace of 2^22 steps is a schedule or geometry bug, not a history (~100
                    // crossings per packet, a few thousand at most): drop the packet with error
                    // ARTES_ERR_RUNAWAY instead of spinning
                    const bool runaway = ncross >= nlim;
                    const bool err31 = !(best < K.inf) | runaway;
                    const bool exit = (w == 0) & side & (nfi == G.nr) & !err31;
                    const bool surf = (w == 0) & (nfi == G.cell_depth) & !err31;
                    bool err = err31 | ((tf == G.cell_depth) & surf);
        #ifdef ARTES_DEBUG
                    {   // the new index of the crossed family must name a cell unless the trace leaves
                        // the grid or reaches the surface (ARTES_ERR_CELL: the packet is dropped before
                        // its out-of-range kappa read, and the run fails)
                        const int nk = !G3D ? G.nr : (w == 0 ? G.nr : (w == 1 ? G.ntheta : G.nphi));
                        if (!err && !exit && !surf && (kn < 0 || kn >= nk)) {
                            log_err(R, ARTES_ERR_CELL);
                            err = true;
                        }
                    }
        #endif
                    // (the error codes are logged on the chain-end paths below: every error stops)
                    auto log_step_err = [&]() {
                        if (runaway) log_err(R, ARTES_ERR_RUNAWAY);
                        log_err(R, err31 ? 31 : 34);
                    };
                    ncross++;
                    const double tau_cell = best * k;
                    const bool prop = (mode == S_PROP);
                    const bool hit = prop && tacc + tau_cell > ttgt;
                    const bool stop = err || exit || surf || hit;
        #ifdef ARTES_DEBUG_LANES
                    dbg_s = stop; dbg_h = prop && hit && !err; dbg_m = !stop; dbg_u = false;
        #endif
                    if constexpr (FLOW) {
                        if (prop && !err && !hit) {   // the segment to the face (ARTES.f90:728-743, 889-904)
                            const int lat = w == 0 ? (side ? 0 : 1) : (w == 1 ? (side ? 2 : 3) : -1);
                            flow_segment(R.flow_g, R.flow_t, cell, tx + best * nx, ty + best * ny, tz + best * nz, nx, ny, nz, best, wI, lat);
                        }
                    }
                    if constexpr (TREL) {
                        // Every lane that crosses -- a move, or a trace end other than an interaction --
                        // takes the crossing's optical depth, trace parameter and face; a move also
                        // takes the new cell.  The trace ends are resolved once per iteration, after the
                        // steps (below): inside every step their branches ran in ~90 % of the steps for
                        // ~4 lanes (a lane that stops sits out the iteration's other steps either way).
                        const bool hitpark = prop & hit & !err;
                        if (!hitpark) {
                            tacc += tau_cell;
                            tpar = best_abs;
                            tf = nfi | (w << 16);
                        }
                        if (!stop) {
                            if constexpr (G3D) {
                                tcr = w == 0 ? kn : tcr;
                                tct = w == 1 ? kn : tct;
                                tcp = w == 2 ? kn : tcp;
                                cell = tcr + (int)__umul24((unsigned)G.nr, (unsigned)tct) + (int)__umul24((unsigned)nrt, (unsigned)tcp);
                            } else {
                                cell += kn - kf;
                                tcr = kn;
                            }
                            load_cell();
                            pending |= 1 << w;
                        } else {
                            // the interaction waits, parked, until enough lanes of the wave need it (the
                            // top of the loop); any other end waits for the end of the iteration
                            parked = hitpark ? 4
                                             : (PK_END | (exit ? PK_EXIT : 0) | (surf ? PK_SURF : 0) | (err31 ? PK_ERR31 : 0) |
                                                (runaway ? PK_RUNAWAY : 0) | (err ? PK_ERR : 0));
                        }
                    } else {
                        if (!stop) {
                            tacc += tau_cell;
                            if constexpr (TREL) {
                                tpar = best_abs;
                            } else {
                                tx = fma(best, nx, tx); ty = fma(best, ny, ty); tz = fma(best, nz, tz);
                            }
                            tf = nfi | (w << 16);
                            if constexpr (G3D) {
                                tcr = w == 0 ? kn : tcr;
                                tct = w == 1 ? kn : tct;
                                tcp = w == 2 ? kn : tcp;
                                cell = tcr + (int)__umul24((unsigned)G.nr, (unsigned)tct) + (int)__umul24((unsigned)nrt, (unsigned)tcp);
                                if constexpr (!TREL) { e0 -= best; e1 -= best; e2 -= best; }
                            } else {
                                cell += kn - kf;
                                tcr = kn;
                            }
                            load_cell();
                            pending |= 1 << w;
                        } else if (prop && !err && hit) {
                            // the interaction in this cell waits, parked, until enough lanes of the
                            // wave need it (the top of the loop)
                            parked = 4;
                        } else if (prop) {
                            if (err) {
                                log_step_err();
                                log_err(R, 3);
                                end = S_END_DROP;
                            } else if (exit) {                             // left the atmosphere
                                end = S_END_EXIT;
                            } else {                                       // reached the surface (ARTES.f90:755-774)
                                // (xi > albedo: absorbed; a black surface absorbs whatever xi is, and
                                // an ended packet's RNG state is not used again, so no draw then)
                                bool absorbed = true;
                                if (R.surface_albedo > 0.0) absorbed = rng.uni() > R.surface_albedo;
                                if (absorbed) {
                                    end = S_END_ABS;
                                } else {
                                    // Lambertian reflection: k_event turns the packet at the surface point,
                                    // the propagation then resumes with the optical depth still to go
                                    const double sf = TREL ? best_abs : best;
                                    px = tx + sf * nx; py = ty + sf * ny; pz = tz + sf * nz;
                                    pcell = pack_cell(tcr, tct, tcp);
                                    pface = pack_face(1, G.cell_depth);
                                    ttgt = ttgt - (tacc + tau_cell);
                                    end = S_SURF_HIT;
                                }
                            }
                        } else {   // a first-optical-depth or peel-off trace reached the boundary
                            tacc += tau_cell;
                            // error codes of the four traces (ARTES.f90:640, 4743, 4549, 4653)
                            if (err) {
                                log_step_err();
                                log_err(R, mode == S_FIRST ? 2 : mode == S_PEEL ? 43 : mode == S_PEEL_T ? 46 : 42);
                            }
                            if (is_peel_trace(mode)) {
                                const int kind = mode == S_PEEL_T ? 1 : mode == S_PEEL_S ? 2 : 0;
                                end = S_PEEL_DONE | (exit ? FLAG_EXIT : 0) | (err ? FLAG_ERR : 0) | (kind << PEEL_KIND_SHIFT);
                            } else if (tacc < 1.e-6 && !surf) {            // forced first interaction (ARTES.f90:658-685)
                                end = S_END_DROP;
                            } else {
                                // the forced first interaction waits (parked, at the chord's far end:
                                // the position, face and cell of the crossing, for a backward walk)
                                // until enough lanes of the wave need it (see the top of the loop)
                                const double sf = TREL ? best_abs : best;
                                tx += sf * nx; ty += sf * ny; tz += sf * nz;
                                tf = nfi | (w << 16);
                                parked = err ? 3 : 1;
                            }
                        }
                    }
                }
            }   // do_step
        }   // have
        }   // rep
        TM_TICK(t3);
        TM_ADD(3, t3 - t2);
        if constexpr (TREL) {
            // The trace ends of this iteration's steps (ARTES.f90:640-656, 745-778, 4743-4761), for
            // every lane that stopped in any of them, once per iteration.  (A surface's albedo draw
            // moves here from the step: the lane draws nothing in between, so its RNG sequence is
            // unchanged.)
            // (the radial-form steps leave the runaway test to here, once per iteration: a trace still
            // stepping past nlim crossings ends as the generic step's runaway does)
            if (have && !parked && !end && ncross >= nlim) parked = PK_END | PK_ERR31 | PK_RUNAWAY | PK_ERR;
            if (__ballot(parked >= PK_END)) {
                if (parked >= PK_END) {
                    int sk = parked;
                    parked = 0;
                    if (sk & PK_RAD) {
                        // the radial-form step (ARTES.f90:2885-3010 faces): the packet crossed sphere tf
                        // (a radial face code): the top sphere is the exit, sphere cell_depth the surface
                        sk |= (tf == G.nr ? PK_EXIT : 0) | (tf == G.cell_depth ? PK_SURF : 0) | ((sk & PK_RAD_E) ? PK_ERR : 0);
                    }
                    const bool exit = (sk & PK_EXIT) != 0, surf = (sk & PK_SURF) != 0, err = (sk & PK_ERR) != 0;
                    if (err) {
                        if (sk & PK_RUNAWAY) log_err(R, ARTES_ERR_RUNAWAY);
                        log_err(R, (sk & PK_ERR31) ? 31 : 34);
                    }
                    if (mode == S_PROP) {
                        if (err) {
                            log_err(R, 3);
                            end = S_END_DROP;
                        } else if (exit) {                             // left the atmosphere
                            end = S_END_EXIT;
                        } else {                                       // reached the surface (ARTES.f90:755-774)
                            // (xi > albedo: absorbed; a black surface absorbs whatever xi is, and
                            // an ended packet's RNG state is not used again, so no draw then)
                            bool absorbed = true;
                            if (R.surface_albedo > 0.0) absorbed = rng.uni() > R.surface_albedo;
                            if (absorbed) {
                                end = S_END_ABS;
                            } else {
                                // Lambertian reflection: k_event turns the packet at the surface point,
                                // the propagation then resumes with the optical depth still to go
                                px = tx + tpar * nx; py = ty + tpar * ny; pz = tz + tpar * nz;
                                pcell = pack_cell(tcr, tct, tcp);
                                pface = pack_face(1, G.cell_depth);
                                ttgt = ttgt - tacc;
                                end = S_SURF_HIT;
                            }
                        }
                    } else {   // a first-optical-depth or peel-off trace reached the boundary
                        // error codes of the four traces (ARTES.f90:640, 4743, 4549, 4653)
                        if (err) log_err(R, mode == S_FIRST ? 2 : mode == S_PEEL ? 43 : mode == S_PEEL_T ? 46 : 42);
                        if (is_peel_trace(mode)) {
                            const int kind = mode == S_PEEL_T ? 1 : mode == S_PEEL_S ? 2 : 0;
                            end = S_PEEL_DONE | (exit ? FLAG_EXIT : 0) | (err ? FLAG_ERR : 0) | (kind << PEEL_KIND_SHIFT);
                        } else if (tacc < 1.e-6 && !surf) {            // forced first interaction (ARTES.f90:658-685)
                            end = S_END_DROP;
                        } else {
                            // the forced first interaction waits (parked, at the chord's far end: the
                            // position, face and cell of the crossing, for a backward walk) until
                            // enough lanes of the wave need it (see the top of the loop)
                            tx += tpar * nx; ty += tpar * ny; tz += tpar * nz;
                            parked = err ? 3 : 1;
                        }
                    }
                }
            }
        }
        if (end) {   // the chain ends: the record now, the list append below or at the next refill
            c_cross += (uint32_t)(ncross - nc0);
            Slot* rec = S.s + slot;
            rec->px = px; rec->py = py; rec->pz = pz;
            rec->r0 = rng.s0; rec->r1 = rng.s1;
            rec->pcell = pcell; rec->pface = pface;
            rec->mode = end; rec->ncross = ncross;
            rec->wI = wI;
            rec->tpeel = tacc;
            rec->ttgt = ttgt;
            pend = end;
            have = false;
        }
        if (!R.late_append) append();
        q_event.flush_if(QFLUSH, L.event, L.event_n);
        q_emit.flush_if(QFLUSH, L.emit, L.emit_n);
        TM_TICK(t4);
        TM_ADD(4, t4 - t3);
        TM_ADD(6, 1);
#ifdef ARTES_DEBUG_LANES
        {
            const unsigned long long bs = __ballot(dbg_s), bh = __ballot(dbg_h), bm = __ballot(dbg_m);
            dbg_anystop += bs != 0; dbg_anyhit += bh != 0; dbg_nstop += __popcll(bs); dbg_nmove += __popcll(bm);
            dbg_nretry += __popcll(__ballot(dbg_r)); dbg_nsetup += __popcll(__ballot(dbg_u));
        }
#endif
    }
    append();
    q_event.flush(L.event, L.event_n);
    q_emit.flush(L.emit, L.emit_n);
    if constexpr (LOOKAHEAD) prefetch_drain();
#ifdef ARTES_DEBUG_TIMING
    {
        TM_TICK(t_end);
        TM_ADD(7, t_end - t_begin);
        __builtin_amdgcn_wave_barrier();
        if ((threadIdx.x & 63) < 20 && (threadIdx.x & 63) != 15) atomicAdd(&R.err[threadIdx.x & 63], my_tm[threadIdx.x & 63]);
    }
#endif
#ifdef ARTES_DEBUG_LANES
    if ((threadIdx.x & 63) == 0) {
        // (development build: error slots reused as counters, the run's error codes are void)
        atomicAdd(&R.err[0], dbg_steps);
        atomicAdd(&R.err[30], dbg_lanes);
        atomicAdd(&R.err[32], dbg_refills);
        atomicAdd(&R.err[40], dbg_tsteps);
        atomicAdd(&R.err[41], dbg_tlanes);
        atomicAdd(&R.err[48], dbg_anystop);
        atomicAdd(&R.err[12], dbg_anyhit);
        atomicAdd(&R.err[1], dbg_nstop);
        atomicAdd(&R.err[2], dbg_nmove);
        atomicAdd(&R.err[4], dbg_nretry);
        atomicAdd(&R.err[5], dbg_nsetup);
        atomicAdd(&R.err[6], dbg_firuns);
        atomicAdd(&R.err[7], dbg_filanes);
        atomicAdd(&R.err[8], dbg_reflanes);
        atomicAdd(&R.err[9], dbg_hruns);
        atomicAdd(&R.err[10], dbg_hlanes);
        atomicAdd(&R.err[17], dbg_f12);
        atomicAdd(&R.err[22], dbg_anyf12);
        atomicAdd(&R.err[23], dbg_f2);
        atomicAdd(&R.err[24], dbg_anyf2);
        atomicAdd(&R.err[49], dbg_rsteps);
        atomicAdd(&R.err[50], dbg_ridle);
        atomicAdd(&R.err[51], dbg_rpark);
        atomicAdd(&R.err[52], dbg_rend);
        atomicAdd(&R.err[53], dbg_rstep);
        atomicAdd(&R.err[54], dbg_rblock);
    }
#endif
    const unsigned long long wv = wave_sum_u64(c_cross), wp = wave_sum_u64(c_peel);
    if ((threadIdx.x & 63) == 0) {
        if (wv) cnt_add(R, ARTES_CNT_CROSSINGS, wv);
        if (wp) cnt_add(R, ARTES_CNT_PEELS, wp);
    }
}

}  // namespace artes
