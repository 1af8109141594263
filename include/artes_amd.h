/*
 * artes_amd.h -- C ABI of the MI355X photon-packet transport engine.
 *
 * This is the drop-in boundary for the reference's hot path: the OpenMP packet
 * loop `radiative_transfer` (ARTES.f90:518-1006) together with the table set-up it
 * consumes (`get_atmosphere` ARTES.f90:2054-2235, `grid_initialize(2)`
 * ARTES.f90:2325-2357) and the per-thread detector reduction (ARTES.f90:957-975).
 * In the reference these are module globals of one Fortran program; here they are
 * a reentrant handle plus plain-pointer calls, so any host (ctypes, cgo, JNI, a
 * Fortran `bind(C)` interface) can drive them.  See INTEGRATION.md.
 *
 * Conventions
 *   - Every array is C-order (row-major) double precision, laid out exactly as the
 *     numpy view of the corresponding atmosphere.fits HDU: FITS axis 1 (the Fortran
 *     first index) is the LAST C index.  E.g. the reference's
 *     cell_scatter_matrix(r,theta,phi,lambda,16,180) (ARTES.f90:2196) is
 *     scatter[180][16][nwav][nphi][ntheta][nr] here.
 *   - Detector tensors are [4][4][ny][nx]: planes 0..2 are the reference's
 *     detector(nx,ny,4,3) (ARTES.f90:84, 2543) in C order -- sum w, sum w^2 (per
 *     peel), peel count -- for Stokes I,Q,U,V; plane 3 is an addition: the
 *     packet-level second moment sum_p (X_p)^2 of each packet's contribution X_p to
 *     the pixel, the honest Monte-Carlo variance (peels of one packet land in the
 *     same pixel, so the per-peel sum w^2 underestimates it by ~1.7-3x).  Values
 *     are in units of packet weight; the caller multiplies by package_energy
 *     (ARTES.f90:964-970).
 *   - totals[ARTES_NUM_TOTALS]: [0..3] sum_p T_p and [4..7] sum_p T_p^2 of each
 *     packet's total detected weight T_p per Stokes component (honest variance of
 *     the integrated photometry); [8] flux_emitted and [9] flux_exit of the thermal
 *     source (ARTES.f90:607, 780, 953), in units of packet weight.
 *   - Peels that carry Stokes I only (thermal emission, ARTES.f90:4519-4598;
 *     Lambertian surface, 4600-4708) add their count to the Stokes-I count alone,
 *     as the reference does.
 *   - Functions return 0 on success or a negative errno-style code; they never
 *     exit the process (the reference calls exit(0) on fatal errors).  A failed
 *     run still reports the counters and totals of the packets it did transport.
 *   - One call at a time per grid handle: the packet pool, the work lists and the
 *     per-call partial counters belong to the handle, so two artes_run_device calls
 *     on one grid from different streams must be ordered by the caller (one stream,
 *     or an event between them).  Separate handles are independent (several engines
 *     can share a device, each on its own stream).
 *   - Error-code counters: uint64_t err[ARTES_NUM_ERR], index = the reference's
 *     "error NNN" number written to error.log (e.g. ARTES.f90:640, 3401).  Two
 *     indices the reference does not use report engine faults, after which the run's
 *     results are invalid and artes_run / artes_run_flow return -5:
 *     ARTES_ERR_WATCHDOG (57) counts waves of the transport kernel stopped by its
 *     iteration watchdog; ARTES_ERR_LISTS (58) counts violations of the work-list
 *     invariants, checked only by ARTES_DEBUG builds ("Work lists").
 *     ARTES_ERR_RUNAWAY (59) counts traces stopped after 2^22 cell crossings (the
 *     packet is dropped and also counted as error 31); ARTES_ERR_GEOM (60) counts
 *     interaction points outside their cell's radial shell, checked only by
 *     ARTES_DEBUG_GEOM builds (a diagnostic: the reference's oblate star emission
 *     produces such points by design).  Two more are trace-state invariants checked
 *     only by ARTES_DEBUG builds, after which the run fails with -5 like 58:
 *     ARTES_ERR_PENDING (61) counts family evaluations of k_trace that clear a
 *     `pending` bit other than the evaluated family's (a bound would then be taken
 *     for an exact face distance), ARTES_ERR_CELL (62) counts cell indices outside
 *     [0, nr) x [0, ntheta) x [0, nphi) after a move or at a trace start (the packet
 *     is dropped before the out-of-range table read).
 */
#ifndef ARTES_AMD_H
#define ARTES_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ARTES_ABI_VERSION 6
#define ARTES_NUM_TOTALS 10
#define ARTES_NUM_ERR 64
#define ARTES_ERR_WATCHDOG 57
#define ARTES_ERR_LISTS 58
#define ARTES_ERR_RUNAWAY 59
#define ARTES_ERR_GEOM 60
#define ARTES_ERR_PENDING 61
#define ARTES_ERR_CELL 62

/* Counter slots (uint64_t counters[ARTES_NUM_COUNTERS]). */
#define ARTES_CNT_CROSSINGS 0   /* cell_face calls (ARTES.f90:2800), all traces   */
#define ARTES_CNT_SCATTERS  1   /* scatter_photon calls (ARTES.f90:1434)          */
#define ARTES_CNT_PEELS     2   /* peel_photon calls (ARTES.f90:4710)             */
#define ARTES_CNT_PACKETS   3   /* packets emitted                                 */
#define ARTES_CNT_EXITED    4   /* packets that left the grid                      */
#define ARTES_CNT_ABSORBED  5   /* surface absorption / roulette / minimum weight  */
#define ARTES_CNT_DROPPED   6   /* cell_error or tau_first < 1e-6 drops            */
#define ARTES_CNT_DETECTED  7   /* peels that reached the detector                 */
#define ARTES_NUM_COUNTERS  8

/* Raw atmosphere as read from atmosphere.fits (ARTES.f90:2067-2198). */
typedef struct artes_grid_desc {
    int32_t nr;              /* radial cells   (faces: nr+1)                       */
    int32_t ntheta;          /* polar cells    (faces: ntheta+1)                   */
    int32_t nphi;            /* azimuthal cells (faces: nphi, 2*pi implicit)       */
    int32_t nwav;            /* wavelengths                                         */
    const double* radial;    /* [nr+1]  m                                           */
    const double* theta_deg; /* [ntheta+1] degrees                                  */
    const double* phi_deg;   /* [nphi] degrees                                      */
    const double* wavelength_um; /* [nwav] micron                                   */
    const double* kappa_sca; /* [nwav][nphi][ntheta][nr]  m^-1                      */
    const double* kappa_abs; /* [nwav][nphi][ntheta][nr]  m^-1                      */
    const double* scatter;   /* [180][16][nwav][nphi][ntheta][nr]                   */
    const double* temperature; /* [nphi][ntheta][nr] K, may be NULL (star source)   */
    double oblateness;       /* planet:oblateness (ARTES.f90:469-471)               */
} artes_grid_desc;

/* Per-call run parameters: the globals radiative_transfer reads. */
typedef struct artes_run_params {
    int32_t wl_index;        /* 0-based wavelength (wl_count-1)                    */
    int32_t nx, ny;          /* detector pixels (1x1 for spectrum/phase)           */
    int32_t photon_source;   /* 1 = star, 2 = planet (thermal emission)            */
    int32_t photon_scattering; /* photon:scattering on/off                         */
    int32_t phase_far;       /* phase_curve && det_phi >= 170 deg (ARTES.f90:1041) */
    int32_t stellar_direction; /* star:direction (ARTES.f90:1080-1111)             */
    int32_t cell_depth;      /* surface face index; <0 => computed (ARTES.f90:2329-2392) */
    double det_theta, det_phi; /* detector direction [rad], already clamped       */
    double x_max, y_max;     /* image half-size [m] (ARTES.f90:475-479)            */
    double fstop;            /* photon:fstop                                        */
    double photon_minimum;   /* photon:minimum                                      */
    double surface_albedo;   /* planet:surface_albedo                               */
    double theta_star, phi_star; /* stellar direction [rad]                         */
    /* thermal source (photon:source=planet), ARTES.f90:1117-1266, 2359-2453 */
    int32_t photon_emission; /* 1 = isotropic, 2 = biased upward (photon:emission)  */
    int32_t thermal_weight;  /* photon:weight: cell luminosity weighting on/off     */
    int32_t ring;            /* planet:ring (thermal cell_depth skips 2 cells)      */
    int32_t packet_moments;  /* 1: also accumulate the packet-level second moments
                              * (detector planes 12-15, totals[4..7]) for honest
                              * Monte-Carlo errors; 0: skip them (the reference has
                              * none, and they double the per-event slot traffic)     */
    double photon_bias;      /* photon:bias, 0 <= b < 1                             */
} artes_run_params;

typedef struct artes_grid artes_grid;

/* ABI / build identification. */
int32_t artes_abi_version(void);
const char* artes_build_info(void);

/* Number of visible devices (hipGetDeviceCount); <0 on error. */
int32_t artes_device_count(void);

/* Build the device-resident tables for one atmosphere on `device`
 * (replaces get_atmosphere post-processing + grid_initialize, ARTES.f90:2172-2270):
 * extinction, albedo (floored at 1e-20), deduplicated scattering matrices with
 * their cumulative sampling tables, p1j integrals and trig face tables. */
int32_t artes_grid_create(const artes_grid_desc* desc, int32_t device, artes_grid** out);
void    artes_grid_destroy(artes_grid* grid);

/* cell_depth for a wavelength (grid_initialize(2), ARTES.f90:2329-2357). */
int32_t artes_grid_cell_depth(const artes_grid* grid, int32_t wl_index);

/* Thermal source tables of one wavelength (grid_initialize(2), planet branch,
 * ARTES.f90:2359-2453, with cell_volume 2274-2300 and planck_function 1350-1367):
 * cell_depth (absorption optical depth 5 from the top; `ring` skips the two outer
 * cells), the total weighted emissivity emissivity_cumulative(nr-1,ntheta-1,nphi-1)
 * [W m-1] that sets package_energy (2535), and optionally cell_luminosity
 * [nphi][ntheta][nr] [W m-1] (the cell_luminosity.fits of write_output, 3658).
 * Needs the temperature array in artes_grid_desc. */
int32_t artes_grid_thermal(artes_grid* grid, int32_t wl_index, int32_t thermal_weight, int32_t ring,
                           int32_t* cell_depth, double* emissivity_total, double* cell_luminosity);

/* Number of distinct (cell, wavelength) scattering matrices kept after dedup. */
int32_t artes_grid_num_matrices(const artes_grid* grid);

/* Run packets [first_packet, first_packet + n_packets) of the global packet
 * sequence keyed by `seed` (one xoroshiro128++ stream per global packet id, so
 * results do not depend on how packets are sharded).  Synchronous; host outputs,
 * all ACCUMULATED into (so shards/wavelengths can be summed in place):
 *   detector   [4][4][ny][nx]   (see Conventions)
 *   totals     [ARTES_NUM_TOTALS] (may be NULL)
 *   counters   [ARTES_NUM_COUNTERS] (may be NULL)
 *   err        [ARTES_NUM_ERR]  (may be NULL)
 * Replaces radiative_transfer's packet loop + thread reduction (ARTES.f90:546-975). */
int32_t artes_run(artes_grid* grid, const artes_run_params* params,
                  uint64_t first_packet, uint64_t n_packets, uint64_t seed,
                  double* detector, double* totals, uint64_t* counters, uint64_t* err);

/* Device variant: outputs are DEVICE pointers (e.g. torch tensors) accumulated
 * into on `stream` (a hipStream_t, NULL = default stream), so the caller can
 * all-reduce `detector_dev` with RCCL on the same stream.  totals_dev holds only
 * the four sum_p T_p^2 values (the sums T_p are the detector plane-0 totals)
 * followed by flux_emitted and flux_exit: totals_dev[6].
 * The event engine polls its live-packet count from the host every few
 * iterations, so the call returns once the transport has drained; the final
 * detector reduction is still in flight on `stream`. */
int32_t artes_run_device(artes_grid* grid, const artes_run_params* params,
                         uint64_t first_packet, uint64_t n_packets, uint64_t seed,
                         double* detector_dev, double* totals_dev, uint64_t* counters_dev,
                         uint64_t* err_dev, void* stream);

/* Energy-transport diagnostics (output:flow_global / output:flow_latitudinal): as
 * artes_run / artes_run_device, plus per-cell accumulators in the reference's
 * cell_flow_global / cell_flow layout with the component fastest (ARTES.f90:81-82,
 * 2311-2322), ACCUMULATED into; either may be NULL (both NULL = plain run):
 *   flow_global      [nphi][ntheta][nr][3]  sum over propagation segments of the
 *                    direction's (r, theta, phi) component at the segment end x segment
 *                    length x Stokes I (add_flow_global, 4992-5011)
 *   flow_latitudinal [nphi][ntheta][nr][4]  Stokes I leaving the cell upward, downward,
 *                    southward (theta increasing), northward (add_flow, 5013-5045)
 * Only propagation segments count (peel-off and first-optical-depth traces do not:
 * 715-743, 874-904).  The host writes flow_global.fits / flow_latitudinal.fits
 * (write_output, 3715-3768).  The device variant takes device pointers. */
int32_t artes_run_flow(artes_grid* grid, const artes_run_params* params,
                       uint64_t first_packet, uint64_t n_packets, uint64_t seed,
                       double* detector, double* totals, uint64_t* counters, uint64_t* err,
                       double* flow_global, double* flow_latitudinal);
int32_t artes_run_device_flow(artes_grid* grid, const artes_run_params* params,
                              uint64_t first_packet, uint64_t n_packets, uint64_t seed,
                              double* detector_dev, double* totals_dev, uint64_t* counters_dev,
                              uint64_t* err_dev, double* flow_global_dev, double* flow_latitudinal_dev,
                              void* stream);

/* Duration in ms of the transport (all launches from emission to drain, without
 * the final detector reduction) of the most recent run on this grid, measured
 * with HIP events on the launch stream (valid once that stream has been
 * synchronised). */
double artes_last_kernel_ms(artes_grid* grid);

/* Per-kernel launch timing (HIP events around every launch on the run's stream).
 * artes_set_profiling(grid, 1) starts recording; artes_kernel_times waits for the
 * recorded launches, writes the summed milliseconds and launch counts per kernel class
 * (ARTES_K_*) and resets the accumulators.  Off by default (no events are recorded). */
#define ARTES_K_TRACE       0   /* k_trace: cell-boundary tracing (the hot loop)      */
#define ARTES_K_EVENT       1   /* k_event: peel-off contribution + scattering       */
#define ARTES_K_EMIT        2   /* k_emit: packet close-out + emission               */
#define ARTES_K_AUX         3   /* list rotation, pool init, detector-copy reduction */
#define ARTES_K_PERSISTENT  4   /* the fused single-kernel engine (tuning "engine" = 1)  */
#define ARTES_NUM_KERNELS   5
int32_t artes_set_profiling(artes_grid* grid, int32_t on);
int32_t artes_kernel_times(artes_grid* grid, double* ms, uint64_t* launches);

/* Debug: per-packet records for packets [first, first+n) (n <= 2^24):
 * rec[n][ARTES_TRACE_FIELDS] = { sum of peeled I weight, scatters, crossings,
 * end state (1 exit, 2 absorbed, 3 dropped), sum of peeled -Q, U, V (the detector's
 * sign convention, ARTES.f90:4953-4960), 0 }.
 * Used by the parity tests to compare trajectories with the CPU oracle. */
#define ARTES_TRACE_FIELDS 8
int32_t artes_run_trace(artes_grid* grid, const artes_run_params* params,
                        uint64_t first_packet, uint64_t n_packets, uint64_t seed,
                        double* records);

/* Schedule tuning of one grid handle (development A/B runs and tests).  `key` names one
 * launch-schedule setting; `value` >= 0 overrides it, -1 restores the default (the measured
 * optimum).  No key except "engine" changes a per-packet result: they move the schedule only.
 * Keys: engine (0 event engine, 1 the fused persistent engine), pool (slots; a pool larger than
 * the setting is reallocated at the next call), steps (k_trace
 * steps per iteration, 4 or 10, 3D grids), refill, static, dgrab, batch, batch_min, hbatch,
 * gbatch, defer, backward, emit_first, late_append, pix1, det_lds, event_lds, event_ldsc,
 * event_block (256 or 768), event_bpc, trace_bpc, wpe (3 or 4), msym, max_it, verbose,
 * trace_gtab (k_trace's face tables in global memory; automatic when they exceed 64 KiB),
 * det_ordered (1: detector planes 0-11 summed as 128-bit fixed-point integers, so identical
 * calls give identical bits; the packet-level moments stay floating-point sums), event_ldsu
 * (0: k_event never stages its tables unpadded)
 * (transport.hip, TUNE).  Returns -22 for an unknown key or a value outside the key's range.
 * The production library reads no environment variable: the reference's drop-in never sees
 * a schedule it did not ask for.  The development build (libartes_hip_dev.so) also takes
 * ARTES_<KEY> from the environment when a grid is created.
 * artes_get_tuning returns the override of `key` (-1: the default) or -22. */
int32_t artes_set_tuning(artes_grid* grid, const char* key, int64_t value);
int64_t artes_get_tuning(const artes_grid* grid, const char* key);

/* The kernel instantiations the last call on this grid launched, e.g.
 * "k_trace<1,0,4,0,8> k_event<1,1,0,768,0>" (template arguments of kernel_trace.hpp /
 * kernel_event.hpp: G3D, OBL, WPE, FLOW, NREP and LDS_T, LDS_D, PIX1, block, LDS_C), or
 * "persistent", or "none" when the call launched no transport kernel (n = 0, or a failure
 * before the first launch); storage owned by the grid, valid until its next call. */
const char* artes_last_launch(artes_grid* grid);

/* Last error message of the calling thread (static storage). */
const char* artes_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* ARTES_AMD_H */
