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

// ---------------------------------------------------- face tables (LDS) ---
// fv[0..nr] = rfront^2, fv[nr+1 .. nr+1+ntheta] = tan^2(theta_f): one array so the
// radial and theta families read their two face values with the same instruction;
// tfl[k] = theta-face flags; phsc[2k], phsc[2k+1] = sin, cos(phi_k)
constexpr int TF_CONE = 1, TF_GT90 = 2, TF_LT90 = 4;

struct TraceTabs {
    const double* fv;
    const double* phsc;
    const int* tfl;
};

__host__ __device__ inline size_t trace_table_bytes(int nr, int ntheta, int nphi) {
    return sizeof(double) * ((size_t)(nr + 1) + (size_t)(ntheta + 1) + 2 * (size_t)nphi) + sizeof(int) * (size_t)(ntheta + 1);
}

__device__ __forceinline__ TraceTabs stage_trace_tables(const DevGrid& G, double* lds) {
    TraceTabs T;
    double* fv = lds;
    for (int i = threadIdx.x; i <= G.nr; i += BLOCK) fv[i] = G.rf2[i];
    for (int i = threadIdx.x; i <= G.ntheta; i += BLOCK) fv[G.nr + 1 + i] = G.tan2[i];
    double* phsc = fv + (G.nr + 1) + (G.ntheta + 1);
    for (int i = threadIdx.x; i < G.nphi; i += BLOCK) { phsc[2 * i] = G.phis[i]; phsc[2 * i + 1] = G.phic[i]; }
    int* tfl = (int*)(phsc + 2 * G.nphi);
    for (int i = threadIdx.x; i <= G.ntheta; i += BLOCK) {
        const double th = G.thetaf[i];
        tfl[i] = (G.tplane[i] == 1 ? TF_CONE : 0) | (th > HALF_PI ? TF_GT90 : 0) | (th < HALF_PI ? TF_LT90 : 0);
    }
    __syncthreads();
    T.fv = fv; T.phsc = phsc; T.tfl = tfl;
    return T;
}

// ------------------------------------------------------- family evaluation ---
// Candidate distances to the inner and outer face of ONE coordinate family of cell
// (cr, ct, cp) from (x, y, z) along n, for a packet sitting on face (ft, fi):
//   fam 0: spheres r_cr, r_cr+1   (ARTES.f90:2885-3010)
//   fam 1: theta cones / the 90-degree plane, faces ct, ct+1 (3014-3290)
//   fam 2: phi half-planes cp, cp+1 (3292-3350)
// 0 = no candidate, as in the reference.  zp = distance to the plane z = 0.
template <bool G3D, bool OBL>
__device__ __forceinline__ void family_candidates(const DevGrid& G, const TraceTabs& T, int fam, double x, double y,
                                                  double z, double n0, double n1, double n2, int ft, int fi, int cr,
                                                  int ct, int cp, double zp, double& d_in, double& d_out) {
    const double ax2 = OBL ? G.ax2 : 1.0, by2 = OBL ? G.by2 : 1.0, cz2 = OBL ? G.cz2 : 1.0;
    const bool isR = !G3D || fam == 0;
    const bool isT = G3D && fam == 1;
    const bool isP = G3D && fam == 2;
    // sphere:  ax2 x^2 + by2 y^2 + cz2 z^2 - r^2        (w = 1,       off = r^2)
    // cone:    ax2 x^2 + by2 y^2 - cz2 z^2 tan^2(theta) (w = -tan^2, off = 0)
    const double Axy = ax2 * n0 * n0 + by2 * n1 * n1, Az = cz2 * n2 * n2;
    const double Bxy = ax2 * x * n0 + by2 * y * n1, Bz = cz2 * z * n2;
    const double Cxy = ax2 * x * x + by2 * y * y, Cz = cz2 * z * z;
    const int kin = isR ? cr : ct;
    const int vb = isR ? 0 : G.nr + 1;
    const double vin = T.fv[vb + kin], vout = T.fv[vb + kin + 1];
    const double win = isR ? 1.0 : -vin, wout = isR ? 1.0 : -vout;
    const double qa0 = Axy + win * Az, qb0 = 2.0 * (Bxy + win * Bz), qc0 = Cxy + win * Cz - (isR ? vin : 0.0);
    const double qa1 = Axy + wout * Az, qb1 = 2.0 * (Bxy + wout * Bz), qc1 = Cxy + wout * Cz - (isR ? vout : 0.0);
    // quadratic_equation (ARTES.f90:4154-4173), both faces
    const double disc0 = qb0 * qb0 - 4.0 * qa0 * qc0, disc1 = qb1 * qb1 - 4.0 * qa1 * qc1;
    const double q0 = -0.5 * (qb0 + copysign(fast_sqrt(disc0), qb0));
    const double q1 = -0.5 * (qb1 + copysign(fast_sqrt(disc1), qb1));
    // phi half-planes: num / den per face (ARTES.f90:3300-3346)
    double num0 = 0.0, den0 = 1.0, num1 = 0.0, den1 = 1.0;
    int pout = 0;
    if constexpr (G3D) {
        const double ga = OBL ? G.a : 1.0, gb = OBL ? G.b : 1.0;
        pout = (cp + 1 == G.nphi) ? 0 : cp + 1;
        const double s0 = T.phsc[2 * cp], c0 = T.phsc[2 * cp + 1];
        const double s1 = T.phsc[2 * pout], c1 = T.phsc[2 * pout + 1];
        den0 = gb * n1 * c0 - ga * n0 * s0; num0 = ga * x * s0 - gb * y * c0;
        den1 = gb * n1 * c1 - ga * n0 * s1; num1 = ga * x * s1 - gb * y * c1;
    }
    // four divisions shared by the families: quadratic roots q/a and c/q, or the two
    // plane intersections num/den
    const double ra0 = fast_div(isP ? num0 : q0, isP ? den0 : qa0);
    const double rb0 = fast_div(qc0, q0);
    const double ra1 = fast_div(isP ? num1 : q1, isP ? den1 : qa1);
    const double rb1 = fast_div(qc1, q1);
    // Per face k (0 inner, 1 outer) the reference's rules reduce to: two roots a_k, b_k
    // (phi planes and the 90-degree plane: one), each a candidate when it exists, lies
    // on the right nappe (cones) and exceeds the face's tolerance; the nearer candidate
    // wins, none if both are equal or the winner is >= 1e100 (quadratic_equation +
    // cell_face root choice, ARTES.f90:2885-3350, 4154-4173); and a per-face veto
    // (same-face and grid-edge rules).  Absent candidates are +inf and the choice is
    // one min, so the wave executes one selection per face instead of one per family
    // and rule.  The phi and 90-degree-plane rules keep their own cap (none) and
    // tolerance (0) exactly.
    const int kout = kin + 1;
    const int kin_f = isP ? cp : kin, kout_f = isP ? pout : kout;
    const int ftype = isR ? 1 : (isT ? 2 : 3);
    const bool same0 = (ft == ftype && fi == kin_f), same1 = (ft == ftype && fi == kout_f);
    const int fl0 = T.tfl[isT ? kin : 0], fl1 = T.tfl[isT ? kout : 0];
    const bool plane0 = isT && !(fl0 & TF_CONE), plane1 = isT && !(fl1 & TF_CONE);
    // roots and their existence
    const bool q_ok0 = disc0 >= 0.0, q_ok1 = disc1 >= 0.0;
    bool va0 = isP ? fabs(den0) > 0.0 : (q_ok0 && fabs(qa0) > 1.e-100);
    bool vb0 = !isP && q_ok0 && fabs(q0) > 1.e-100;
    bool va1 = isP ? fabs(den1) > 0.0 : (q_ok1 && fabs(qa1) > 1.e-100);
    bool vb1 = !isP && q_ok1 && fabs(q1) > 1.e-100;
    // cone nappe filter (ARTES.f90:3040-3064): a root on the other nappe is no crossing
    // (the reference's `s > 1e-15` guard is implied by the tolerance test below)
    if (isT) {
        const bool gt0 = fl0 & TF_GT90, lt0 = fl0 & TF_LT90, gt1 = fl1 & TF_GT90, lt1 = fl1 & TF_LT90;
        const double za0 = fma(ra0, n2, z), zb0 = fma(rb0, n2, z), za1 = fma(ra1, n2, z), zb1 = fma(rb1, n2, z);
        va0 = va0 && !((za0 > 0.0 && gt0) || (za0 < 0.0 && lt0));
        vb0 = vb0 && !((zb0 > 0.0 && gt0) || (zb0 < 0.0 && lt0));
        va1 = va1 && !((za1 > 0.0 && gt1) || (za1 < 0.0 && lt1));
        vb1 = vb1 && !((zb1 > 0.0 && gt1) || (zb1 < 0.0 && lt1));
    }
    // the 90-degree plane: one root at zp, moving towards it (ARTES.f90:3066-3070, 3116-3118)
    const double a0 = plane0 ? zp : ra0, a1 = plane1 ? zp : ra1;
    if (plane0) { va0 = n2 > 1.e-15; vb0 = false; }
    if (plane1) { va1 = n2 < -1.e-15; vb1 = false; }
    // tolerances: re-crossing the face the packet sits on needs 1e-3 m (spheres: outer
    // face only, cones: both; ARTES.f90:2944, 3157), 1e-15 otherwise, 0 for the plane
    const double tol0 = plane0 ? 0.0 : ((same0 && isT) ? 1.e-3 : 1.e-15);
    const double tol1 = plane1 ? 0.0 : ((same1 && !isP) ? 1.e-3 : 1.e-15);
    va0 = va0 && a0 > tol0; vb0 = vb0 && rb0 > tol0;
    va1 = va1 && a1 > tol1; vb1 = vb1 && rb1 > tol1;
    // vetoes
    //   spheres: the inner sphere the packet sits on (ARTES.f90:2899-2960)
    //   theta:   the grid's polar faces; a cone the packet sits on unless the root lies
    //            beyond the apex side it faces; the plane it sits on (3014-3290)
    //   phi:     the half-plane the packet sits on; the outer one also when the inner
    //            face's root is >= 1e100 (sic: sp0, ARTES.f90:3318, 3346)
    const bool sp0_big = !(same0) && fabs(den0) > 0.0 && !(ra0 < 1.e100);
    const bool kill0 = isR ? same0
                     : isT ? (ct == 0 || (same0 && (plane0 || !(fl0 & TF_GT90))))
                           : same0;
    const bool kill1 = isR ? false
                     : isT ? (kout == G.ntheta || (same1 && (plane1 || !(fl1 & TF_LT90))))
                           : (same1 || sp0_big);
    constexpr double INF = __builtin_inf();
    const double m0 = fmin(va0 ? a0 : INF, vb0 ? rb0 : INF);
    const double m1 = fmin(va1 ? a1 : INF, vb1 ? rb1 : INF);
    const bool z0 = kill0 || (va0 && vb0 && a0 == rb0) || !(m0 < 1.e100);
    const bool z1 = kill1 || (va1 && vb1 && a1 == rb1) || !(m1 < 1.e100);
    d_in = z0 ? 0.0 : m0;
    d_out = z1 ? 0.0 : m1;
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
// FLOW instantiations add the energy-transport diagnostics to propagation segments.
template <bool G3D, bool OBL, int WPE, bool FLOW = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_trace(DevGrid G, DevRun R, Pool S, Lists L) {
    extern __shared__ double s_tab[];
    const TraceTabs T = stage_trace_tables(G, s_tab);
    const int n = *L.trace_in_n;
    const int split = *L.trace_in_split;   // [0, split): new packets' traces; then k_event's, stored backwards
    const int home = blockIdx.x & 7;
    __shared__ int s_q[2][BLOCK];
    const int wbase = threadIdx.x & ~63;
    WaveQueue q_event{&s_q[0][wbase], 0}, q_emit{&s_q[1][wbase], 0};
    TraceCursor cur = make_cursor(n, R.static_q64);
    const int fam_all = !G3D ? 1 : (G.nphi > 1 ? 7 : 3);
    constexpr double NONE = -1.e300;
    bool have = false;
#ifdef ARTES_DEBUG_LANES
    unsigned long long dbg_steps = 0, dbg_lanes = 0, dbg_refills = 0, dbg_tsteps = 0, dbg_tlanes = 0;
#endif
    // packet state (slot line 0) and trace state
    int slot = -1, mode = 0, pcell = 0, pface = 0, ncross = 0;
    double px = 0, py = 0, pz = 0, ttgt = 0, wI = 0;
    Rng rng{0, 0};
    int tcr = 0, tct = 0, tcp = 0, tft = 0, tfi = 0, pending = 0;
    double tx = 0, ty = 0, tz = 0, nx = 0, ny = 0, nz = 0, tacc = 0, tpar = 0, inz = 0;
    // per family (radial, theta, phi) the nearest face ahead as a trace parameter, and its
    // side (bit f of `sides`: 0 inner, 1 outer face)
    double m0 = NONE, m1 = NONE, m2 = NONE;
    int sides = 0;
    uint32_t c_cross = 0, c_peel = 0;
    // backward propagation after the forced first interaction (see the FIRST-trace end).
    // During a first trace: the packet's crossings when it started.  During the backward
    // trace that may follow: 2 x crossings at its start + the first trace's steps + 1
    // (from which the forward walk's step count follows at the interaction).  0 otherwise.
    int kb = 0;
    int parked = 0;   // 1: waiting for the batched forced first interaction (3: after a cell error)

    // a trace starts at the packet position with zero optical depth
    auto start_trace = [&](double d0, double d1, double d2) {
        tx = px; ty = py; tz = pz;
        unpack_cell(pcell, tcr, tct, tcp);
        unpack_face(pface, tft, tfi);
        nx = d0; ny = d1; nz = d2;
        tacc = 0.0;
        tpar = 0.0;
        pending = fam_all;
        if constexpr (G3D) inz = fast_rcp(nz);
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
        // where the first trace stopped (tx, tft, tfi: set when the lane parked) to optical
        // depth tau_first - tau.  Same cells in reverse, so the same interaction point up to
        // rounding; crossing counts are kept as the forward walk's (kb).  Not with the flow
        // diagnostics (segment order).
        bool back = false;
        if constexpr (!FLOW) back = R.backward && mid && !err && tau_first - tau < tau;
        kb = back ? 2 * ncross + (ncross - kb) + 1 : 0;
        if (back) {
            ttgt = fmax(tau_first - tau, 0.0);   // tau rounds to <= tau_first + 1 ulp
            nx = -nx; ny = -ny; nz = -nz;
            tacc = 0.0;
            tpar = 0.0;
            pending = fam_all;
            if constexpr (G3D) inz = fast_rcp(nz);
        } else {
            ttgt = tau;
            start_trace(nx, ny, nz);
        }
    };

    for (;;) {
        {
            const unsigned long long pk = __ballot(parked != 0);
            if (pk) {
                const int stepping = __popcll(__ballot(have && parked == 0));
                if (__popcll(pk) >= R.batch || stepping < R.batch_min || cur.exhausted) {
                    if (parked) {
                        first_interaction(parked & 2);
                        parked = 0;
                    }
                }
            }
        }
        // ---------------------------------------------------------------- refill
        if (!cur.exhausted) {
            const unsigned long long idle = __ballot(!have);
            if (__popcll(idle) >= R.refill || idle == __ballot(true)) {
                const int my = wave_take(cur, L.grab, home, !have);
#ifdef ARTES_DEBUG_LANES
                dbg_refills++;
#endif
                if (!have && my >= 0) slot = L.trace_in[my < split ? my : S.P - 1 - (my - split)];
                if (!have && my >= 0 && slot >= 0) {   // -1: a hole left by a dropped or retired packet
                    const Slot* rec = S.s + slot;
                    mode = rec->mode;
                    px = rec->px; py = rec->py; pz = rec->pz;
                    const double ldx = rec->dx, ldy = rec->dy, ldz = rec->dz;
                    ttgt = rec->ttgt;
                    rng.s0 = rec->r0; rng.s1 = rec->r1;
                    pcell = rec->pcell; pface = rec->pface;
                    ncross = rec->ncross;
                    wI = rec->wI;
                    const bool peel = is_peel_trace(mode);
                    start_trace(peel ? R.det0 : ldx, peel ? R.det1 : ldy, peel ? R.det2 : ldz);
                    have = true;
                    kb = (mode == S_FIRST) ? ncross : 0;
                }
            }
        }
        if (!__any(have) && cur.exhausted) break;   // (all lanes idle otherwise: every grab was a hole)
#ifdef ARTES_DEBUG_LANES
        dbg_steps++;
        dbg_lanes += __popcll(__ballot(have));
        if (cur.exhausted) { dbg_tsteps++; dbg_tlanes += __popcll(__ballot(have)); }
#endif
        int end = 0;   // 0: continue, else the slot's new mode
        if (have && !parked) {
            // extinction and albedo of the current cell: issued first so the L2 round trip
            // overlaps the face evaluation (the cell is known before the step)
            const int cell = tcr + G.nr * (tct + G.ntheta * tcp);
            // one 16-byte load at a 32-bit byte offset (ncell < 2^28, checked at grid creation)
            const double2 kv = *(const double2*)((const char*)G.ka + ((unsigned)cell << 4));
            const double k = kv.x;
            const double alb = kv.y;
            // ------------------------------------------- evaluate one face family
            const int fam = G3D ? __builtin_ctz(pending) : 0;
            double din, dout;
            family_candidates<G3D, OBL>(G, T, fam, tx, ty, tz, nx, ny, nz, tft, tfi, tcr, tct, tcp, -tz * inz, din, dout);
            // the evaluated family's nearest face ahead goes to the cache: the other face of a
            // family only matters while the packet sits on the first (and then the family
            // is evaluated again)
            const bool uo = dout > 0.0 && !(din > 0.0 && din <= dout);
            const double dm = uo ? dout : din;
            const double tm = dm > 0.0 ? tpar + dm : NONE;
            if (fam == 0) m0 = tm;
            if constexpr (G3D) {
                if (fam == 1) m1 = tm;
                if (fam == 2) m2 = tm;
            }
            sides = (sides & ~(1 << fam)) | ((uo ? 1 : 0) << fam);
            pending &= pending - 1;
            if (pending == 0) {
                // ------------------------------------------------ trace step
                // candidates: both faces of the family just evaluated (exact distances) and
                // the cached nearest face of each other family; `which` = family + 3 * side
                double e0 = -1.0, e1 = -1.0, e2 = -1.0;
                if constexpr (G3D) {
                    e0 = fam == 0 ? -1.0 : m0 - tpar;
                    e1 = fam == 1 ? -1.0 : m1 - tpar;
                    e2 = fam == 2 ? -1.0 : m2 - tpar;
                }
                // nearest face, 'large' then 'small' solutions (ARTES.f90:3358-3418)
                double best = 1.e100;
                int which = -1;
#define ARTES_CONSIDER(dd, w, thr) if ((dd) > (thr) && (dd) < best) { best = (dd); which = (w); }
#define ARTES_PASS(thr)                                                                    \
                ARTES_CONSIDER(din, fam, thr)                                              \
                ARTES_CONSIDER(dout, fam + 3, thr)                                         \
                if constexpr (G3D) {                                                       \
                    ARTES_CONSIDER(e0, 0 + 3 * (sides & 1), thr)                           \
                    ARTES_CONSIDER(e1, 1 + 3 * ((sides >> 1) & 1), thr)                    \
                    ARTES_CONSIDER(e2, 2 + 3 * ((sides >> 2) & 1), thr)                    \
                }
                ARTES_PASS(1.e-9)
                if (which < 0) {
                    best = 1.e100;
                    ARTES_PASS(1.e-12)
                }
#undef ARTES_PASS
#undef ARTES_CONSIDER
                // next_cell (ARTES.f90:2671-2798)
                int nft = 0, nfi = -999, ncr = tcr, nct = tct, ncp = tcp;
                bool err = false;
                switch (which) {
                    case 0: nft = 1; nfi = tcr; ncr = tcr - 1; break;
                    case 3: nft = 1; nfi = tcr + 1; ncr = tcr + 1; break;
                    case 1: nft = 2; nfi = tct; nct = tct - 1; break;
                    case 4: nft = 2; nfi = tct + 1; nct = tct + 1; break;
                    case 2: nft = 3; nfi = tcp; ncp = (tcp == 0) ? G.nphi - 1 : tcp - 1; break;
                    case 5: nft = 3; { const int po = (tcp + 1 == G.nphi) ? 0 : tcp + 1; nfi = po; ncp = po; } break;
                    default: err = true; log_err(R, 31); break;
                }
                const bool exit = (nft == 1 && nfi == G.nr);
                if (tft == 1 && tfi == G.cell_depth && nft == 1 && nfi == G.cell_depth) { err = true; log_err(R, 34); }
                if (ncr < 0) ncr = 0;
                c_cross++;
                ncross++;
                const double tau_cell = best * k;
                const bool surf = (nft == 1 && nfi == G.cell_depth);
                const bool prop = (mode == S_PROP);
                const bool hit = prop && tacc + tau_cell > ttgt;
                const bool stop = err || exit || surf || hit;
                if constexpr (FLOW) {
                    if (prop && !err && !hit) {   // the segment to the face (ARTES.f90:728-743, 889-904)
                        const int lat = which == 3 ? 0 : which == 0 ? 1 : which == 4 ? 2 : which == 1 ? 3 : -1;
                        flow_segment(R.flow_g, R.flow_t, cell, tx + best * nx, ty + best * ny, tz + best * nz, nx, ny, nz, best, wI, lat);
                    }
                }
                if (!stop) {
                    tacc += tau_cell;
                    tx += best * nx; ty += best * ny; tz += best * nz;
                    tpar += best;
                    tft = nft; tfi = nfi; tcr = ncr; tct = nct; tcp = ncp;
                    pending = 1 << (which % 3);
                } else if (prop && !err && hit) {
                    // interaction in this cell (ARTES.f90:705-720), then the scattering-loop
                    // head (788-813): roulette, albedo weight, minimum weight
                    const double s = fast_div(ttgt - tacc, k);
                    px = tx + s * nx; py = ty + s * ny; pz = tz + s * nz;
                    pcell = pack_cell(tcr, tct, tcp);
                    pface = 0;
                    if (kb) {   // a backward trace: count the steps the forward one takes
                        c_cross += (uint32_t)(kb - 2 * ncross);
                        ncross = kb - ncross;
                        kb = 0;
                    }
                    if constexpr (FLOW) flow_segment(R.flow_g, R.flow_t, cell, px, py, pz, nx, ny, nz, s, wI, -1);   // (715, 874)
                    const double xi = rng.uni();   // a killed packet's RNG state is not used again
                    bool kill = !R.photon_scattering || xi < R.fstop;
                    if (alb < 1.0 && alb > 0.0) wI *= alb / (1.0 - R.fstop);
                    kill = kill || wI <= R.pmin;
                    if (kill) {
                        end = S_END_ABS;
                    } else {                                       // peel-off trace (ARTES.f90:4722-4761)
                        c_peel++;
                        mode = S_PEEL;
                        start_trace(R.det0, R.det1, R.det2);
                    }
                } else if (prop) {
                    if (err) {
                        log_err(R, 3);
                        end = S_END_DROP;
                    } else if (exit) {                             // left the atmosphere
                        end = S_END_EXIT;
                    } else {                                       // reached the surface (ARTES.f90:755-774)
                        const double xi = rng.uni();
                        if (xi > R.surface_albedo) {
                            end = S_END_ABS;
                        } else {
                            // Lambertian reflection: k_event turns the packet at the surface point,
                            // the propagation then resumes with the optical depth still to go
                            px = tx + best * nx; py = ty + best * ny; pz = tz + best * nz;
                            pcell = pack_cell(tcr, tct, tcp);
                            pface = pack_face(1, G.cell_depth);
                            ttgt = ttgt - (tacc + tau_cell);
                            end = S_SURF_HIT;
                        }
                    }
                } else {   // a first-optical-depth or peel-off trace reached the boundary
                    tacc += tau_cell;
                    // error codes of the four traces (ARTES.f90:640, 4743, 4549, 4653)
                    if (err) log_err(R, mode == S_FIRST ? 2 : mode == S_PEEL ? 43 : mode == S_PEEL_T ? 46 : 42);
                    if (is_peel_trace(mode)) {
                        const int kind = mode == S_PEEL_T ? 1 : mode == S_PEEL_S ? 2 : 0;
                        end = S_PEEL_DONE | (exit ? FLAG_EXIT : 0) | (err ? FLAG_ERR : 0) | (kind << PEEL_KIND_SHIFT);
                    } else if (tacc < 1.e-6 && !surf) {            // forced first interaction (ARTES.f90:658-685)
                        end = S_END_DROP;
                    } else {
                        // the forced first interaction waits (parked, at the chord's far end)
                        // until enough lanes of the wave need it (see the top of the loop)
                        tx += best * nx; ty += best * ny; tz += best * nz;
                        tft = nft; tfi = nfi;
                        parked = err ? 3 : 1;
                    }
                }
                if (end) {   // write the packet state back once
                    Slot* rec = S.s + slot;
                    rec->px = px; rec->py = py; rec->pz = pz;
                    rec->r0 = rng.s0; rec->r1 = rng.s1;
                    rec->pcell = pcell; rec->pface = pface;
                    rec->mode = end; rec->ncross = ncross;
                    rec->wI = wI;
                    rec->tpeel = tacc;
                    rec->ttgt = ttgt;
                    have = false;
                }
            }   // pending == 0
        }   // have
        q_event.push(end && to_event_list(end), slot, L.event, L.event_n);
        q_emit.push(end && !to_event_list(end), slot, L.emit, L.emit_n);
    }
    q_event.flush(L.event, L.event_n);
    q_emit.flush(L.emit, L.emit_n);
#ifdef ARTES_DEBUG_LANES
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&R.err[60], dbg_steps);
        atomicAdd(&R.err[61], dbg_lanes);
        atomicAdd(&R.err[59], dbg_refills);
        atomicAdd(&R.err[54], dbg_tsteps);
        atomicAdd(&R.err[55], dbg_tlanes);
    }
#endif
    const unsigned long long w = wave_sum_u64(c_cross), wp = wave_sum_u64(c_peel);
    if ((threadIdx.x & 63) == 0) {
        if (w) atomicAdd(&R.cnt[ARTES_CNT_CROSSINGS], w);
        if (wp) atomicAdd(&R.cnt[ARTES_CNT_PEELS], wp);
    }
}

}  // namespace artes
