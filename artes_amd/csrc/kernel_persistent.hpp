// kernel_persistent.hpp -- the fused single-kernel engine ("persistent"): one packet
// per lane for its whole life, a per-lane state machine whose hot state is one trace
// step, with the rare peel/scatter event deferred until R.defer lanes of the wave need
// it.  Kept as the reference design the event engine (kernel_event.hpp) is measured
// against; selected with ARTES_ENGINE=persistent.
#pragma once

#include "device_common.hpp"

namespace artes {

template <bool G3D, bool TRACE>
__global__ __launch_bounds__(BLOCK) void transport_kernel(DevGrid G, DevRun R) {
    const uint64_t nthreads = (uint64_t)gridDim.x * BLOCK;
    uint64_t next = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;   // static interleaved share
    double* __restrict__ det = R.det + (size_t)(blockIdx.x % R.ncopy) * R.det_stride;
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
                    interp_matrix(P, false, acos(mu), sc);
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
                    double c2b_unused, s2b_unused;
                    sample_angles(G, R, G.cums + (size_t)m * CUM_DOUBLES, rng, st, alpha, beta, c2b_unused, s2b_unused);
                    double e0, e1, e2;
                    direction_cosine(R, alpha, beta, dx, dy, dz, e0, e1, e2);
                    double sc[16];
                    interp_matrix(G.mats + (size_t)m * MAT_DOUBLES, false, acos(alpha), sc);
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
                if constexpr (TRACE) {   // s_pt holds the packet's peeled I, -Q, U, V totals
                    double* rr = R.rec + (size_t)(pid - R.first) * ARTES_TRACE_FIELDS;
                    rr[0] = rec_peel; rr[1] = (double)rec_scat; rr[2] = (double)rec_cross; rr[3] = (double)endst;
                    rr[4] = s_pt[1][lane]; rr[5] = s_pt[2][lane]; rr[6] = s_pt[3][lane]; rr[7] = 0.0;
                    rec_peel = 0.0; rec_scat = 0; rec_cross = 0;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double t = s_pt[k][lane];
                    if (t != 0.0) atomicAdd(&s_tot2[k], t * t);
                    s_pt[k][lane] = 0.0;
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
                        else { mode = M_NEW; endst = E_DROPPED; }   // (unreachable: launch() rejects surface reflection for this engine)
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
    if (lane < ARTES_NUM_COUNTERS) cnt_add(R, lane, s_cnt[lane]);
    if (lane < 4) tot_add(R, lane, s_tot2[lane]);
}

}  // namespace artes
