// Test-only library (libartes_unit.so, not part of the product path): runs single device
// functions of the engine on given inputs, so tests can compare them with the reference's
// angle-based forms near their branch boundaries (tests/test_gpu_unit_checks.py).
//
//   artes_unit_scatter_geometry: azimuth_cs + direction_cosine_cs (k_event's scattering,
//     ARTES.f90:1962-2052) and peel_rotation (k_event's peel-off, 4864-4920) per case.
//
// Not declared in include/artes_amd.h: the drop-in boundary does not contain it.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstring>

#include "device_common.hpp"

namespace artes {

// per case in[9]: incoming direction d (3), direction_cosine's alpha, beta, Stokes st (4)
// per case out[8]: new direction e (3), the peel's Stokes so (4), flags (bit 0: peel made,
// bit 1: drop)
__global__ void k_unit_scatter_geometry(DevRun R, const double* __restrict__ in, const double* __restrict__ sc_in,
                                        double* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* c = in + (size_t)i * 9;
    const double dx = c[0], dy = c[1], dz = c[2];
    double cpo, spo;
    azimuth_cs(dx, dy, cpo, spo);
    double e0, e1, e2;
    direction_cosine_cs(R, c[3], c[4], dx, dy, dz, cpo, spo, e0, e1, e2);
    double st[4] = {c[5], c[6], c[7], c[8]}, sc[16], so[4] = {0, 0, 0, 0};
    for (int k = 0; k < 16; k++) sc[k] = sc_in[k];
    double mu = dx * R.det0 + dy * R.det1 + dz * R.det2;   // (as k_event: ARTES.f90:4770-4776)
    if (mu >= 1.0) mu = 1.0 - 1.e-10;
    else if (mu <= -1.0) mu = -1.0 + 1.e-10;
    bool drop = false;
    const bool made = peel_rotation(R, dz, mu, cpo, spo, st, sc, so, drop);
    double* o = out + (size_t)i * 8;
    o[0] = e0; o[1] = e1; o[2] = e2;
    o[3] = so[0]; o[4] = so[1]; o[5] = so[2]; o[6] = so[3];
    o[7] = (made ? 1.0 : 0.0) + (drop ? 2.0 : 0.0);
}

}  // namespace artes

using namespace artes;

// n cases; the detector direction (det_theta, det_phi) set up as artes_run's (transport.hip);
// sc16: the 4x4 matrix applied by the peel; err[64]: the error codes logged.  0, or a
// negative HIP failure.
extern "C" int artes_unit_scatter_geometry(const double* in, int n, double det_theta, double det_phi, const double* sc16,
                                           double* out, unsigned long long* err) {
    if (n <= 0) return 0;
    DevRun R;
    std::memset(&R, 0, sizeof(R));
    R.det0 = sin(det_theta) * cos(det_phi);
    R.det1 = sin(det_theta) * sin(det_phi);
    R.det2 = cos(det_theta);
    R.det_phi = atan2(R.det1, R.det0);
    if (R.det_phi < 0.0) R.det_phi += 2.0 * M_PI;
    if (R.det_phi > 2.0 * M_PI) R.det_phi -= 2.0 * M_PI;
    R.cdphi = cos(R.det_phi); R.sdphi = sin(R.det_phi);
    double *d_in = nullptr, *d_out = nullptr, *d_sc = nullptr;
    unsigned long long* d_err = nullptr;
    int rc = 0;
    const size_t nin = (size_t)n * 9 * sizeof(double), nout = (size_t)n * 8 * sizeof(double);
    if (hipMalloc(&d_in, nin) != hipSuccess || hipMalloc(&d_out, nout) != hipSuccess ||
        hipMalloc(&d_sc, 16 * sizeof(double)) != hipSuccess || hipMalloc(&d_err, 64 * sizeof(unsigned long long)) != hipSuccess) {
        rc = -2;
    } else if (hipMemcpy(d_in, in, nin, hipMemcpyHostToDevice) != hipSuccess ||
               hipMemcpy(d_sc, sc16, 16 * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
               hipMemset(d_err, 0, 64 * sizeof(unsigned long long)) != hipSuccess) {
        rc = -3;
    } else {
        R.err = d_err;
        hipLaunchKernelGGL(k_unit_scatter_geometry, dim3((n + 255) / 256), dim3(256), 0, 0, R, d_in, d_sc, d_out, n);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = -4;
        else if (hipMemcpy(out, d_out, nout, hipMemcpyDeviceToHost) != hipSuccess ||
                 hipMemcpy(err, d_err, 64 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
            rc = -3;
    }
    hipFree(d_in); hipFree(d_out); hipFree(d_sc); hipFree(d_err);
    return rc;
}
