// tables.hpp -- host-side table construction for the transport engine.
//
// Replaces the table work of the reference's get_atmosphere / grid_initialize
// (ARTES.f90:2097-2235, 2247-2270, 2329-2357) and adds what the GPU design needs:
//   * extinction kappa = kappa_sca + kappa_abs and albedo floored at 1e-20 (ARTES.f90:2178-2188)
//   * per-(wavelength, cell) scattering matrices deduplicated into a small table
//     of unique matrices (a 32x16x32 uniform atmosphere has ONE), each stored
//     angle-major [180][16] so the interpolation at one angle is two contiguous
//     128-byte rows (the reference's cell_scatter_matrix(r,t,p,l,16,180) layout puts
//     them 16*ncell*nwav doubles apart, ARTES.f90:2196)
//   * per unique matrix the cumulative theta-sampling tables
//     A_j(i) = sum_{k<=i} P_1j(k) sin(beta_k) pi/180   (j = 1..4, i = 0..180)
//     so scattering_angle_sampling's 180-bin scan (ARTES.f90:1610-1656) becomes a
//     binary search over a linear combination of four tables: the same CDF, so the
//     same distribution; p1j_int = A_j(180) (ARTES.f90:2203-2230)
//   * the cumulative azimuth tables SC2(i) = sum cos2beta, SS2(i) = sum sin2beta
//     (ARTES.f90:404-420, 1545-1587)
//   * face tables: rfront^2, tan^2(theta_f), thetaplane, sin/cos(phi_f) (ARTES.f90:2261-2270)
//   * thermal source (build_thermal): per wavelength the absorption cell_depth, cell
//     luminosity weights and the emissivity CDF of the planet branch of
//     grid_initialize(2) (ARTES.f90:2359-2453), laid out in the reference's sampling
//     order so emit_photon's linear scan (1126-1154) becomes a binary search
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/artes_amd.h"

namespace artes {

constexpr int NANG = 180;
constexpr int NELEM = 16;
constexpr int MAT_DOUBLES = NANG * NELEM;       // 2880
constexpr int CUM_DOUBLES = (NANG + 1) * 4;     // 724

struct HostTables {
    int nr = 0, ntheta = 0, nphi = 0, nwav = 0, ncell = 0;
    double oblate_x = 1.0, oblate_y = 1.0, oblate_z = 1.0;
    std::vector<double> rfront, rf2, thetaf, tan2, phif, phis, phic;
    std::vector<int32_t> tplane;
    std::vector<double> kappa;     // [nwav][ncell]
    std::vector<double> kabs;      // [nwav][ncell] absorption (thermal source)
    std::vector<double> temperature;  // [ncell], empty if not given
    std::vector<double> wavelength;   // [nwav] m
    std::vector<double> tcos;      // cos(theta_f) [ntheta+1]
    std::vector<double> albedo;    // [nwav][ncell]
    std::vector<int32_t> matid;    // [nwav][ncell]
    std::vector<double> mats;      // [nmat][180][16]
    std::vector<double> cums;      // [nmat][181][4]
    std::vector<double> sc2, ss2;  // [181]
    std::vector<int32_t> cell_depth;  // [nwav], star branch
    int nmat = 0;
};

static inline uint64_t fnv_mix(uint64_t h, uint64_t v) {
    h ^= v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
    return h * 0x100000001b3ULL;
}

inline HostTables build_tables(const artes_grid_desc& d) {
    HostTables T;
    if (d.nr < 1 || d.ntheta < 1 || d.nphi < 1 || d.nwav < 1) throw std::invalid_argument("grid dimensions must be >= 1");
    if (!d.radial || !d.theta_deg || !d.phi_deg || !d.kappa_sca || !d.kappa_abs || !d.scatter)
        throw std::invalid_argument("null array in artes_grid_desc");
    const double pi = 4.0 * std::atan(1.0);
    T.nr = d.nr; T.ntheta = d.ntheta; T.nphi = d.nphi; T.nwav = d.nwav;
    T.ncell = d.nr * d.ntheta * d.nphi;
    T.oblate_x = 1.0 / (1.0 - d.oblateness);   // ARTES.f90:469-471
    T.oblate_y = T.oblate_x;
    T.oblate_z = 1.0;

    T.rfront.assign(d.radial, d.radial + d.nr + 1);
    T.rf2.resize(d.nr + 1);
    for (int i = 0; i <= d.nr; i++) T.rf2[i] = T.rfront[i] * T.rfront[i];
    for (int i = 1; i <= d.nr; i++)
        if (!(T.rfront[i] > T.rfront[i - 1])) throw std::invalid_argument("radial faces must increase");

    T.thetaf.resize(d.ntheta + 1); T.tan2.resize(d.ntheta + 1); T.tplane.resize(d.ntheta + 1);
    for (int i = 0; i <= d.ntheta; i++) {       // ARTES.f90:2097-2106, 2261-2264
        double t = d.theta_deg[i];
        T.tplane[i] = (t < 90.0 - 1.e-6 || t > 90.0 + 1.e-6) ? 1 : 2;
        T.thetaf[i] = t * pi / 180.0;
        double tt = std::tan(T.thetaf[i]);
        T.tan2[i] = tt * tt;
    }
    T.tcos.resize(d.ntheta + 1);
    for (int i = 0; i <= d.ntheta; i++) T.tcos[i] = std::cos(T.thetaf[i]);   // theta_grid_cos, ARTES.f90:2263
    T.phif.resize(d.nphi); T.phis.resize(d.nphi); T.phic.resize(d.nphi);
    for (int i = 0; i < d.nphi; i++) {          // ARTES.f90:2267-2270
        T.phif[i] = d.phi_deg[i] * pi / 180.0;
        T.phic[i] = std::cos(T.phif[i]);
        T.phis[i] = std::sin(T.phif[i]);
    }

    const size_t nwc = (size_t)d.nwav * T.ncell;
    T.kabs.assign(d.kappa_abs, d.kappa_abs + nwc);
    if (d.temperature) T.temperature.assign(d.temperature, d.temperature + T.ncell);
    T.wavelength.resize(d.nwav);
    for (int i = 0; i < d.nwav; i++) T.wavelength[i] = d.wavelength_um ? d.wavelength_um[i] * 1.e-6 : 0.0;
    T.kappa.resize(nwc); T.albedo.resize(nwc);
    for (size_t i = 0; i < nwc; i++) {           // ARTES.f90:2178-2188
        double ext = d.kappa_sca[i] + d.kappa_abs[i];
        double alb = 0.0;
        if (ext > 0.0) alb = d.kappa_sca[i] / ext;
        if (alb < 1.e-20) alb = 1.e-20;
        T.kappa[i] = ext;
        T.albedo[i] = alb;
    }

    // --- matrix dedup: hash every (wl, cell) matrix streaming plane by plane ---
    // scatter index: ((a*16 + e)*nwav + wl)*ncell + cell, a = angle, e = element
    std::vector<uint64_t> h(nwc, 1469598103934665603ULL);
    for (int a = 0; a < NANG; a++)
        for (int e = 0; e < NELEM; e++) {
            const double* plane = d.scatter + ((size_t)(a * NELEM + e)) * nwc;
            for (size_t i = 0; i < nwc; i++) {
                uint64_t bits;
                std::memcpy(&bits, &plane[i], 8);
                h[i] = fnv_mix(h[i], bits);
            }
        }
    auto same = [&](size_t i, size_t j) {
        for (int a = 0; a < NANG; a++)
            for (int e = 0; e < NELEM; e++) {
                const double* plane = d.scatter + ((size_t)(a * NELEM + e)) * nwc;
                if (std::memcmp(&plane[i], &plane[j], 8) != 0) return false;
            }
        return true;
    };
    std::vector<size_t> rep;                                     // unique id -> representative index
    T.matid.resize(nwc);
    {   // fast path: assign by hash, then verify every element in one streaming pass
        std::unordered_map<uint64_t, int32_t> first;
        for (size_t i = 0; i < nwc; i++) {
            auto it = first.find(h[i]);
            if (it == first.end()) {
                int32_t id = (int32_t)rep.size();
                first.emplace(h[i], id);
                rep.push_back(i);
                T.matid[i] = id;
            } else {
                T.matid[i] = it->second;
            }
        }
        bool collision = false;
        for (int a = 0; a < NANG && !collision; a++)
            for (int e = 0; e < NELEM && !collision; e++) {
                const double* plane = d.scatter + ((size_t)(a * NELEM + e)) * nwc;
                for (size_t i = 0; i < nwc; i++)
                    if (std::memcmp(&plane[i], &plane[rep[T.matid[i]]], 8) != 0) { collision = true; break; }
            }
        if (collision) {   // slow exact path (hash collision): bucket by hash, compare element-wise
            rep.clear();
            std::unordered_map<uint64_t, std::vector<int32_t>> buckets;
            for (size_t i = 0; i < nwc; i++) {
                auto& ids = buckets[h[i]];
                int32_t found = -1;
                for (int32_t id : ids)
                    if (same(rep[id], i)) { found = id; break; }
                if (found < 0) {
                    found = (int32_t)rep.size();
                    rep.push_back(i);
                    ids.push_back(found);
                }
                T.matid[i] = found;
            }
        }
    }
    T.nmat = (int)rep.size();
    T.mats.resize((size_t)T.nmat * MAT_DOUBLES);
    for (int m = 0; m < T.nmat; m++)
        for (int a = 0; a < NANG; a++)
            for (int e = 0; e < NELEM; e++)
                T.mats[(size_t)m * MAT_DOUBLES + a * NELEM + e] = d.scatter[((size_t)(a * NELEM + e)) * nwc + rep[m]];

    // sinbeta(n) and (cos|sin)2beta(n) bin averages, 1-based (ARTES.f90:409-420)
    double sinb[NANG + 1], c2b[NANG + 1], s2b[NANG + 1];
    for (int i = 1; i <= NANG; i++) {
        sinb[i] = (std::sin((double)i * pi / 180.0) + std::sin((double)(i - 1) * pi / 180.0)) / 2.0;
        c2b[i] = (std::cos(2.0 * (double)i * pi / 180.0) + std::cos(2.0 * (double)(i - 1) * pi / 180.0)) / 2.0;
        s2b[i] = (std::sin(2.0 * (double)i * pi / 180.0) + std::sin(2.0 * (double)(i - 1) * pi / 180.0)) / 2.0;
    }
    T.cums.assign((size_t)T.nmat * CUM_DOUBLES, 0.0);
    for (int m = 0; m < T.nmat; m++) {
        double* C = &T.cums[(size_t)m * CUM_DOUBLES];
        const double* P = &T.mats[(size_t)m * MAT_DOUBLES];
        for (int j = 0; j < 4; j++) C[j] = 0.0;
        for (int i = 1; i <= NANG; i++)
            for (int j = 0; j < 4; j++)
                C[i * 4 + j] = C[(i - 1) * 4 + j] + P[(i - 1) * NELEM + j] * sinb[i] * pi / 180.0;
    }
    T.sc2.assign(NANG + 1, 0.0);
    T.ss2.assign(NANG + 1, 0.0);
    for (int i = 1; i <= NANG; i++) {
        T.sc2[i] = T.sc2[i - 1] + c2b[i];
        T.ss2[i] = T.ss2[i - 1] + s2b[i];
    }

    // cell_depth per wavelength, star branch (ARTES.f90:2329-2357)
    T.cell_depth.resize(d.nwav);
    for (int wl = 0; wl < d.nwav; wl++) {
        int cell_max = 1000000, depth = 0;
        for (int j = 0; j < d.ntheta; j++)
            for (int k = 0; k < d.nphi; k++) {
                double tot = 0.0;
                for (int i = 0; i < d.nr; i++) {
                    int r = d.nr - i - 1;
                    size_t c = (size_t)wl * T.ncell + ((size_t)k * d.ntheta + j) * d.nr + r;
                    tot += T.kappa[c] * (T.rfront[d.nr - i] - T.rfront[d.nr - i - 1]);
                    depth = r;
                    if (tot > 30.0) break;
                }
                if (depth < cell_max) cell_max = depth;
            }
        T.cell_depth[wl] = cell_max;
    }
    return T;
}

// Thermal source of one wavelength (grid_initialize(2), planet branch, ARTES.f90:2359-2453).
struct ThermalTables {
    int cell_depth = 0;
    double total = 0.0;              // emissivity_cumulative(nr-1, ntheta-1, nphi-1) [W m-1]
    std::vector<double> cdf;         // [(nr - cell_depth) * ntheta * nphi], order (i, j, k), k fastest
    std::vector<double> weight;      // cell_weight [ncell] (C order [nphi][ntheta][nr])
    std::vector<double> luminosity;  // cell_luminosity [ncell] [W m-1]
};

inline ThermalTables build_thermal(const HostTables& T, int wl, bool thermal_weight, bool ring) {
    if (T.temperature.empty()) throw std::invalid_argument("photon:source=planet needs the temperature array");
    const double pi = 4.0 * std::atan(1.0);
    const double k_b = 1.3806488e-23, hh = 6.62606957e-34, cc = 2.99792458e8;   // ARTES.f90:10-13
    const double lam = T.wavelength[wl];
    const double* ab = &T.kabs[(size_t)wl * T.ncell];
    auto cidx = [&](int i, int j, int k) { return ((size_t)k * T.ntheta + j) * T.nr + i; };
    // planck_function, per steradian (ARTES.f90:1362)
    auto planck = [&](double t) { return (2.0 * hh * cc * cc / std::pow(lam, 5.0)) / (std::exp(hh * cc / (lam * k_b * t)) - 1.0); };
    // cell_volume (ARTES.f90:2274-2300)
    auto volume = [&](int i, int j, int k) {
        double dphi = 2.0 * pi;
        if (T.nphi > 1) dphi = (k < T.nphi - 1) ? T.phif[k + 1] - T.phif[k] : 2.0 * pi - T.phif[k];
        const double r1 = T.rfront[i + 1], r0 = T.rfront[i];
        return T.oblate_x * T.oblate_y * T.oblate_z * (1.0 / 3.0) * (r1 * r1 * r1 - r0 * r0 * r0) * (T.tcos[j] - T.tcos[j + 1]) * dphi;
    };
    ThermalTables X;
    // deepest cell where the absorption optical depth from the top exceeds 5 (ARTES.f90:2361-2391)
    int cell_max = 1000000, depth = 0;
    const int grid_out = ring ? 2 : 0;
    for (int j = 0; j < T.ntheta; j++)
        for (int k = 0; k < T.nphi; k++) {
            double tot = 0.0;
            for (int i = grid_out; i < T.nr; i++) {
                tot += ab[cidx(T.nr - i - 1, j, k)] * (T.rfront[T.nr - i] - T.rfront[T.nr - i - 1]);
                depth = T.nr - i - 1;
                if (tot > 5.0) break;
            }
            if (depth < cell_max) cell_max = depth;
        }
    X.cell_depth = cell_max;
    double norm = 0.0;
    for (int i = X.cell_depth; i < T.nr; i++)
        for (int j = 0; j < T.ntheta; j++)
            for (int k = 0; k < T.nphi; k++) {
                const size_t c = cidx(i, j, k);
                if (T.temperature[c] > 0.0) norm += ab[c] * planck(T.temperature[c]) * volume(i, j, k);
            }
    X.weight.assign(T.ncell, 0.0);
    X.luminosity.assign(T.ncell, 0.0);
    X.cdf.assign((size_t)(T.nr - X.cell_depth) * T.ntheta * T.nphi, 0.0);
    double total = 0.0;
    size_t o = 0;
    for (int i = X.cell_depth; i < T.nr; i++)
        for (int j = 0; j < T.ntheta; j++)
            for (int k = 0; k < T.nphi; k++, o++) {
                const size_t c = cidx(i, j, k);
                if (T.temperature[c] > 0.0 && ab[c] > 0.0) {
                    const double b = planck(T.temperature[c]), v = volume(i, j, k);
                    X.weight[c] = thermal_weight ? norm / (v * ab[c] * b) : 1.0;
                    X.luminosity[c] = 4.0 * pi * v * ab[c] * b;
                    total = total + X.luminosity[c] * X.weight[c];
                }
                X.cdf[o] = total;
            }
    X.total = total;
    return X;
}

}  // namespace artes
