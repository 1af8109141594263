// transport.hip -- MI355X (gfx950) photon-packet transport engine + C ABI.
//
// The hot path of the reference, `radiative_transfer` (ARTES.f90:518-1006), runs here as
// an EVENT ENGINE over a pool of in-flight packets in HBM (a 128-byte transport record
// and a 128-byte diagnostic record per slot, kernel_event.hpp): one host iteration launches
//   k_trace  (kernel_trace.hpp) every cell_face step (ARTES.f90:2800-3470) of the first
//            optical depth, propagation and peel-off traces, one packet per lane, lanes
//            refilling themselves from the trace list;
//   k_event  peel-off contribution + scattering (ARTES.f90:4765-4984, 819-846);
//   k_emit   packet close-out + emission of new packets (ARTES.f90:546-597, 1027-1268);
//   k_rotate list rotation;
// and the host polls the live-packet count every few iterations until the pool drains.
// The fused single-kernel engine of the first design (kernel_persistent.hpp) is kept as
// ARTES_ENGINE=persistent for comparison tests only.
//
// All arithmetic is FP64 (the reference is double precision; the cell-face quadratics
// cancel ~15 digits at R ~ 7e7 m).  Tables: tables.hpp.  Detector: planes
// 0-8 accumulated per k_event block in LDS and flushed into privatised HBM copies
// (copy = blockIdx % ncopy, det_copies), summed by reduce_detector.  No MFMA: this is branchy
// per-packet work, not a contraction.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "device_common.hpp"
#include "kernel_persistent.hpp"

// k_trace's step slots per loop iteration on fine 3D and radial-only grids (the coarse 3D grids'
// 4: ARTES_COARSE_NREP): 10 since the fused radial step -- bench +1.1 %, ray3d / hg / iso k_trace
// -1.3 / -2.1 / -1.2 % against 8; 9, 11 and 12 slower (profiles/r06/ab/trace_nrep_sweep_*.txt)
#ifndef ARTES_FINE_NREP
#define ARTES_FINE_NREP 10
#endif
#include "kernel_event.hpp"
#include "kernel_trace.hpp"

namespace artes {

// add the CNT_COPIES partial event counters of a call (cnt_add) into the caller's counters
__global__ void sum_counters(const unsigned long long* __restrict__ part, unsigned long long* __restrict__ out,
                             const double* __restrict__ tpart, double* __restrict__ tout) {
    const int k = threadIdx.x;
    if (k < ARTES_NUM_COUNTERS) {
        unsigned long long s = 0;
#pragma unroll
        for (int c = 0; c < CNT_COPIES; c++) s += part[c * CNT_STRIDE + k];
        out[k] += s;
    } else if (k >= 32 && k < 32 + 6) {   // the totals' six sums
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < CNT_COPIES; c++) s += tpart[c * CNT_STRIDE + k - 32];
        tout[k - 32] += s;
    }
}

// how many privatised detector copies a call uses: the blocks of a launch flush into them
// with device-scope atomics, which the memory side serialises per line (a k_event block adds
// its LDS detector at its end, a one-pixel wave its ten sums), so more copies, fewer blocks
// per line: 64 while they fit in 64 MiB, at least 8
static int det_copies(size_t stride) {
    int n = NCOPY_MAX;
    while (n > 8 && stride * n * sizeof(double) > ((size_t)64 << 20)) n >>= 1;
    return n;
}

// sum the ncopy privatised detectors into `out` ([4][4][ny][nx], accumulated).  Copy
// plane 8 counts the polarised peels, copy plane 9 the I-only ones (thermal emission,
// surface): the reference adds the first to the counts of all four Stokes components
// (ARTES.f90:4969-4972), the second to the count of I alone (4581, 4688)
__global__ void reduce_detector(const double* __restrict__ copies, size_t stride, int ncopy, size_t plane, double* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 16 * plane) return;
    double s = 0.0;
    for (int c = 0; c < ncopy; c++) s += copies[(size_t)c * stride + i];
    const size_t slot = i / plane;           // 0..15 = moment*4 + stokes
    if (slot == 8) {
        const size_t pix = i - 8 * plane;
        double s9 = 0.0;
        for (int c = 0; c < ncopy; c++) s9 += copies[(size_t)c * stride + 9 * plane + pix];
        out[i] += s + s9;
        out[9 * plane + pix] += s;
        out[10 * plane + pix] += s;
        out[11 * plane + pix] += s;
    } else if (slot == 9 || slot == 10 || slot == 11) {
        // filled from slots 8 and 9
    } else {
        out[i] += s;
    }
}

// det_ordered (kernel_event.hpp, fix_add): the nfix fixed-point copies of planes 0-9 summed in
// 128-bit integers (exact, so in any order) and converted once, into copy 0 of the floating-point
// detector (whose planes 0-9 nothing else writes then): reduce_detector then adds zeros to it
__global__ void reduce_fixed(const unsigned long long* __restrict__ fix, size_t fix_stride, int nfix, size_t plane,
                             double* __restrict__ copy0) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 10 * plane) return;
    unsigned long long lo = 0, hi = 0;
    for (int c = 0; c < nfix; c++) {
        const unsigned long long l = fix[(size_t)c * fix_stride + 2 * i], h = fix[(size_t)c * fix_stride + 2 * i + 1];
        const unsigned long long s = lo + l;
        hi += h + (s < lo ? 1ull : 0ull);
        lo = s;
    }
    const bool neg = (long long)hi < 0;
    if (neg) {
        hi = ~hi + (lo == 0 ? 1ull : 0ull);
        lo = 0ull - lo;
    }
    const double v = (double)hi * 0x1p-16 + (double)lo * 0x1p-80;
    copy0[i] = neg ? -v : v;
}

}  // namespace artes

// ================================================================= C ABI ===
using namespace artes;

// ----------------------------------------------------------- schedule tuning ---
// Launch-schedule overrides of one grid handle (artes_set_tuning).  Every default below is
// the measured optimum, and no key except `engine` changes a per-packet result: they move
// the schedule only (tests/test_gpu_engine.py).  The production library takes them through
// that call alone -- it reads no environment variable, so a stray variable in a user's shell
// cannot change the schedule or the engine.  The development build (-DARTES_DEV_KNOBS,
// libartes_hip_dev.so, and the ARTES_DEBUG test build) also takes ARTES_<KEY> from the
// environment at grid creation, for the A/B tools under tools/.
enum TuneKey : int {
    T_ENGINE, T_POOL, T_STEPS, T_REFILL, T_STATIC, T_DGRAB, T_BATCH, T_BATCH_MIN, T_HBATCH, T_GBATCH, T_DEFER,
    T_BACKWARD, T_EMIT_FIRST, T_LATE_APPEND, T_PIX1, T_DET_LDS, T_EVENT_LDS, T_EVENT_LDSC, T_EVENT_BLOCK, T_EVENT_BPC,
    T_TRACE_BPC, T_WPE, T_MSYM, T_MAX_IT, T_VERBOSE, T_TRACE_GTAB, T_DET_ORDERED, T_EVENT_LDSU, T_NUM
};
struct TuneSpec {
    const char* name;
    long long lo, hi;   // accepted range ("steps": 4 or 8; "event_block": 256 or 768)
};
static const TuneSpec TUNE[T_NUM] = {
    {"engine", 0, 1},            // 0 the event engine, 1 the fused persistent engine (comparison tests)
    {"pool", 1024, 1LL << 26},   // packet-pool slots (default 131072 per CU)
    {"steps", 4, 16},            // k_trace steps per loop iteration on 3D grids: 4 or ARTES_FINE_NREP (10)
    {"refill", 1, 64},           // k_trace: refill a wave once this many lanes are idle
    {"static", 0, 64},           // statically dealt share of the trace list, in 1/64
    {"dgrab", 1, 4096},          // least list entries of a dynamic grab
    {"batch", 1, 64},            // batched forced first interaction: lanes that wait
    {"batch_min", 1, 64},        // ... or fewer than this many lanes still step
    {"hbatch", 1, 64},           // batched interaction + peel set-up: lanes that wait
    {"gbatch", 1, 64},           // batched theta evaluations: lanes that wait (the 4-step k_trace)
    {"defer", 1, 64},            // persistent engine: event deferral
    {"backward", 0, 1},          // backward walk after the forced first interaction
    {"emit_first", 0, 1},        // trace-list order
    {"late_append", 0, 1},       // list appends of ended chains at the wave's next refill
    {"pix1", 0, 1},              // one-pixel detectors: per-lane sums
    {"det_lds", 0, 1},           // k_event detector in LDS
    {"event_lds", 0, 1},         // k_event scattering tables in LDS
    {"event_ldsc", 0, 1},        // k_event cumulative tables alone in LDS
    {"event_block", 256, 768},   // k_event block: 256 or 768 threads
    {"event_bpc", 1, 16},        // k_event blocks per CU (LDS-detector kernels)
    {"trace_bpc", 1, 16},        // k_trace blocks per CU
    {"wpe", 3, 4},               // k_trace occupancy target (waves per SIMD)
    {"msym", 0, 1},              // block-diagonal matrices read as 4 elements per row
    {"max_it", 1, 1LL << 40},    // engine iterations before a call fails
    {"verbose", 0, 1},           // one stderr line per call (pool, iterations, kernel choice)
    {"trace_gtab", 0, 1},        // k_trace's face tables in global memory (automatic beyond 64 KiB)
    {"det_ordered", 0, 1},       // detector partials summed in a fixed order: bit-reproducible images
    {"event_ldsu", 0, 1},        // k_event tables in LDS unpadded when only that fits
};

struct artes_grid {
    int device = 0;
    long long tune[T_NUM];   // -1: the default (artes_set_tuning)
    artes_grid() { std::fill(tune, tune + T_NUM, -1LL); }
    HostTables T;
    double *d_rf2 = nullptr, *d_thetaf = nullptr, *d_tan2 = nullptr, *d_phif = nullptr, *d_phis = nullptr,
           *d_phic = nullptr, *d_kappa = nullptr, *d_albedo = nullptr, *d_ka = nullptr, *d_mats = nullptr, *d_cums = nullptr,
           *d_sc2 = nullptr, *d_ss2 = nullptr;
    double ka_fstop = -1.0;   // the fstop d_ka's gamma column was built for (launch); -1: not yet
    int *d_tplane = nullptr, *d_matid = nullptr;
    double *d_rfront = nullptr, *d_tcos = nullptr;
    double *d_th_cdf = nullptr, *d_th_weight = nullptr;   // thermal tables of the last planet-source call
    size_t th_cap = 0;
    double* d_copies = nullptr;
    size_t copies_cap = 0;
    double* d_out = nullptr;          // scratch outputs for the host-pointer variant
    size_t out_cap = 0;
    double* d_tot = nullptr;
    unsigned long long* d_cnt = nullptr;
    unsigned long long* d_cnt_part = nullptr;   // [CNT_COPIES][CNT_STRIDE] per-call partial counters (cnt_add)
    double* d_tot_part = nullptr;                // [CNT_COPIES][CNT_STRIDE] per-call partial totals (tot_add)
    unsigned long long* d_err = nullptr;
    double* d_rec = nullptr;
    size_t rec_cap = 0;
    double* d_flow = nullptr;         // scratch flow accumulators of the host-pointer variant [7][ncell]
    double* d_ttab = nullptr;         // k_trace's face tables in global memory (GTAB kernels)
    size_t ttab_cap = 0;
    unsigned long long* d_fix = nullptr;   // det_ordered: fixed-point detector copies
    size_t fix_cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    int max_blocks = 0;
    int num_cus = 0;
    // event engine: packet pool + work lists (allocated on first use)
    Pool pool{};
    void* pool_mem = nullptr;
    int* d_lists[2] = {nullptr, nullptr};
    int* d_event = nullptr;
    int* d_emit = nullptr;
    int* d_counts = nullptr;              // [field][NSUB], CPAD apart (cnt_at): [0],[1] trace lists, [2] event, [3] emit, [4],[5] splits, [8] debug iteration
    int* d_owner = nullptr;               // ARTES_DEBUG: [P] slot ownership tags
    unsigned int* d_grab = nullptr;       // [NSUB][8] shard cursors, CPAD apart (grab_at)
    unsigned long long* d_next = nullptr;
    int* h_count = nullptr;               // pinned
    hipEvent_t ev_poll = nullptr;
    int trace_blocks = 0;
    int trace_nrep = 0;                   // steps per iteration of the last k_trace launched
    std::string last_trace, last_event;   // the kernel instantiations of the last call (artes_last_launch)
    int last_engine = 0;                  // the last call's engine: 0 none launched, 1 event, 2 persistent
    std::string launch_info;
    long long last_iterations = 0;
    // occupancy answers per (kernel, dynamic LDS bytes), queried once per grid
    std::vector<std::pair<std::pair<const void*, size_t>, int>> occ;
    // the scattering matrices of one wavelength, renumbered (wl_set): a call reads only its
    // wavelength's matrices, so k_event's LDS budget is spent on those alone
    struct WlSet {
        int nmat = -1;
        double* d_mats = nullptr;   // [nmat][180][16]
        double* d_mats4 = nullptr;  // [nmat][180][4] (P11, P12, P33, P34) when every matrix is block-diagonal symmetric
        double* d_cums = nullptr;   // [nmat][181][4]
        int* d_matid = nullptr;     // [ncell] local ids
    };
    std::vector<WlSet> wl;
    // per-launch timing (artes_set_profiling)
    bool prof = false;
    std::vector<hipEvent_t> prof_ev;     // start/end pairs
    std::vector<int> prof_kind;
    std::vector<int> prof_start;         // per launch: the index in prof_ev of its start event
    size_t prof_used = 0;
    // inside the engine's iteration loop the launches follow each other on the stream with nothing
    // in between (until the live-count poll), so a launch starts at the previous launch's end event:
    // one event per launch instead of two (the bench's profiled step: 904 -> 899 ms with none at all)
    bool prof_loop = false, prof_chain = false;
};

// a tuning value of the handle, or `def` when it was not set
static long long tv(const artes_grid* g, int k, long long def) { return g->tune[k] >= 0 ? g->tune[k] : def; }

#ifdef ARTES_DEV_KNOBS
// development build: ARTES_<KEY> from the environment at grid creation (ARTES_ENGINE=persistent)
static void tuning_from_env(artes_grid* g) {
    for (int k = 0; k < T_NUM; k++) {
        std::string var = "ARTES_";
        for (const char* c = TUNE[k].name; *c; c++) var += (char)toupper(*c);
        const char* e = getenv(var.c_str());
        if (!e) continue;
        const long long v = k == T_ENGINE ? (std::string(e) == "persistent" ? 1 : 0) : atoll(e);
        g->tune[k] = std::max(TUNE[k].lo, std::min(TUNE[k].hi, v));
        if (k == T_STEPS) g->tune[k] = v == 4 ? 4 : ARTES_FINE_NREP;
        if (k == T_EVENT_BLOCK) g->tune[k] = v == 256 ? 256 : 768;
    }
}
#endif

// resident blocks per CU of `kernel` at `lds` bytes of dynamic LDS (cached per grid: the
// event engine launches the same few kernels hundreds of times per call)
template <class K>
static int blocks_per_cu(artes_grid* g, K kernel, size_t lds, int block = BLOCK) {
    const std::pair<const void*, size_t> key{(const void*)kernel, lds};
    for (const auto& e : g->occ)
        if (e.first == key) return e.second;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds) != hipSuccess) per_cu = 1;
    per_cu = std::max(1, per_cu);
    g->occ.push_back({key, per_cu});
    return per_cu;
}

// run `launch` between two recorded events when profiling is on
template <class F>
static void timed(artes_grid* g, int kind, hipStream_t s, F&& launch) {
    if (!g->prof) { launch(); return; }
    const size_t i = g->prof_used;
    while (g->prof_ev.size() < 2 * (i + 1)) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) { launch(); return; }
        g->prof_ev.push_back(e);
    }
    if (g->prof_kind.size() < i + 1) g->prof_kind.resize(i + 1);
    if (g->prof_start.size() < i + 1) g->prof_start.resize(i + 1);
    int si = (int)(2 * i);
    if (g->prof_loop && g->prof_chain && i > 0) si = (int)(2 * (i - 1) + 1);   // (the previous launch's end)
    else hipEventRecord(g->prof_ev[2 * i], s);
    launch();
    hipEventRecord(g->prof_ev[2 * i + 1], s);
    g->prof_kind[i] = kind;
    g->prof_start[i] = si;
    g->prof_used = i + 1;
    g->prof_chain = true;
}

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
#ifdef ARTES_DEV_KNOBS
    return "artes_amd transport engine: gfx950 HIP, FP64, event engine (k_trace / k_event / k_emit); "
           "development build: tuning also from ARTES_* environment variables";
#else
    return "artes_amd transport engine: gfx950 HIP, FP64, event engine (k_trace / k_event / k_emit)";
#endif
}

int32_t artes_set_tuning(artes_grid* g, const char* key, int64_t value) {
    if (!g || !key) return fail(-22, "null argument");
    for (int k = 0; k < T_NUM; k++) {
        if (std::strcmp(key, TUNE[k].name) != 0) continue;
        if (value < 0) { g->tune[k] = -1; return 0; }   // back to the default
        if (value < TUNE[k].lo || value > TUNE[k].hi || (k == T_STEPS && value != 4 && value != ARTES_FINE_NREP) ||
            (k == T_EVENT_BLOCK && value != 256 && value != 768))
            return fail(-22, std::string("tuning value out of range for ") + key);
        if (k == T_STEPS && !(g->T.ntheta > 1 || g->T.nphi > 1) && value != ARTES_FINE_NREP)
            return fail(-22, "steps: radial-only grids have the fine-grid k_trace only (" + std::to_string(ARTES_FINE_NREP) + " steps)");
        g->tune[k] = value;
        return 0;
    }
    return fail(-22, std::string("unknown tuning key ") + key);
}

int64_t artes_get_tuning(const artes_grid* g, const char* key) {
    if (!g || !key) return -22;
    for (int k = 0; k < T_NUM; k++)
        if (std::strcmp(key, TUNE[k].name) == 0) return g->tune[k];
    return -22;
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
    void* ptrs[] = {g->d_rf2, g->d_thetaf, g->d_tan2, g->d_phif, g->d_phis, g->d_phic, g->d_kappa, g->d_albedo, g->d_ka,
                    g->d_mats, g->d_cums, g->d_sc2, g->d_ss2, g->d_tplane, g->d_matid, g->d_copies, g->d_out,
                    g->d_tot, g->d_cnt, g->d_cnt_part, g->d_tot_part, g->d_err, g->d_rec, g->d_rfront, g->d_tcos, g->d_th_cdf, g->d_th_weight,
                    g->d_flow, g->d_ttab};
    for (void* p : ptrs)
        if (p) hipFree(p);
    void* eptrs[] = {g->pool_mem, g->d_lists[0], g->d_lists[1], g->d_event, g->d_emit, g->d_counts, g->d_grab, g->d_next,
                     g->d_owner, g->d_fix};
    for (void* p : eptrs)
        if (p) hipFree(p);
    for (auto& W : g->wl) {
        if (W.d_mats) hipFree(W.d_mats);
        if (W.d_mats4) hipFree(W.d_mats4);
        if (W.d_cums) hipFree(W.d_cums);
        if (W.d_matid) hipFree(W.d_matid);
    }
    if (g->h_count) hipHostFree(g->h_count);
    if (g->ev_poll) hipEventDestroy(g->ev_poll);
    for (hipEvent_t e : g->prof_ev) hipEventDestroy(e);
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
    // (k_trace's fused radial step leaves out the 1e100 caps of the radial roots, which no
    // grid below 1e40 m can reach: kernel_trace.hpp, radial_next)
    if (!(g->T.rfront[g->T.nr] < 1.e40)) return fail(-22, "radial grid beyond 1e40 m");
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
    HIP_TRY(hipMalloc((void**)&g->d_ka, 2 * T.kappa.size() * sizeof(double)));   // (filled by launch: ka_table)
    HIP_TRY(upload(&g->d_sc2, T.sc2));
    HIP_TRY(upload(&g->d_ss2, T.ss2));
    HIP_TRY(upload(&g->d_rfront, T.rfront));
    HIP_TRY(upload(&g->d_tcos, T.tcos));
    HIP_TRY(hipMalloc((void**)&g->d_tot, 6 * sizeof(double)));
    HIP_TRY(hipMalloc((void**)&g->d_cnt, ARTES_NUM_COUNTERS * sizeof(unsigned long long)));
    HIP_TRY(hipMalloc((void**)&g->d_cnt_part, CNT_COPIES * CNT_STRIDE * sizeof(unsigned long long)));
    HIP_TRY(hipMalloc((void**)&g->d_tot_part, CNT_COPIES * CNT_STRIDE * sizeof(double)));
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
    g->num_cus = prop.multiProcessorCount;
    HIP_TRY(hipDeviceSynchronize());
#ifdef ARTES_DEV_KNOBS
    tuning_from_env(g.get());
#endif
    *out = g.release();
    return 0;
}

int32_t artes_grid_cell_depth(const artes_grid* g, int32_t wl) {
    if (!g || wl < 0 || wl >= g->T.nwav) return -22;
    return g->T.cell_depth[wl];
}

int32_t artes_grid_num_matrices(const artes_grid* g) { return g ? g->T.nmat : -22; }

int32_t artes_grid_thermal(artes_grid* g, int32_t wl, int32_t thermal_weight, int32_t ring, int32_t* cell_depth,
                           double* emissivity_total, double* cell_luminosity) {
    if (!g || wl < 0 || wl >= g->T.nwav) return fail(-22, "bad grid or wavelength index");
    try {
        const ThermalTables X = build_thermal(g->T, wl, thermal_weight != 0, ring != 0);
        if (cell_depth) *cell_depth = X.cell_depth;
        if (emissivity_total) *emissivity_total = X.total;
        if (cell_luminosity) std::memcpy(cell_luminosity, X.luminosity.data(), X.luminosity.size() * sizeof(double));
    } catch (const std::exception& e) {
        return fail(-22, e.what());
    }
    return 0;
}

}  // extern "C"

// the matrices wavelength `wl` uses, renumbered in order of first use over the cells, with
// their cumulative tables and the per-cell local ids (built on the first call at `wl`)
static int32_t wl_set(artes_grid* g, int wl, artes_grid::WlSet** out) {
    if (g->wl.empty()) g->wl.resize(g->T.nwav);
    artes_grid::WlSet& W = g->wl[wl];
    if (W.nmat < 0) {
        const HostTables& T = g->T;
        const size_t nc = (size_t)T.ncell;
        std::vector<int> loc((size_t)T.nmat, -1), ids;
        std::vector<int32_t> matid(nc);
        for (size_t c = 0; c < nc; c++) {
            const int gid = T.matid[(size_t)wl * nc + c];
            if (loc[gid] < 0) { loc[gid] = (int)ids.size(); ids.push_back(gid); }
            matid[c] = loc[gid];
        }
        std::vector<double> mats(ids.size() * MAT_DOUBLES), cums(ids.size() * CUM_DOUBLES);
        for (size_t k = 0; k < ids.size(); k++) {
            std::memcpy(&mats[k * MAT_DOUBLES], &T.mats[(size_t)ids[k] * MAT_DOUBLES], MAT_DOUBLES * sizeof(double));
            std::memcpy(&cums[k * CUM_DOUBLES], &T.cums[(size_t)ids[k] * CUM_DOUBLES], CUM_DOUBLES * sizeof(double));
        }
        HIP_TRY(upload(&W.d_mats, mats));
        HIP_TRY(upload(&W.d_cums, cums));
        // the block-diagonal form of spheres and Rayleigh scattering, value by value (interp_matrix):
        // k_event then reads 4 of the 16 elements per row (built whenever the matrices qualify;
        // launch() reads ARTES_MSYM=0 per call to use the 16-element form instead)
        bool sym = true;
        for (size_t k = 0; k < mats.size() && sym; k += NELEM) {
            const double* m = &mats[k];
            sym = m[2] == 0.0 && m[3] == 0.0 && m[6] == 0.0 && m[7] == 0.0 && m[8] == 0.0 && m[9] == 0.0 && m[12] == 0.0 &&
                  m[13] == 0.0 && m[4] == m[1] && m[5] == m[0] && m[15] == m[10] && m[14] == -m[11];
        }
        if (sym) {
            std::vector<double> m4(ids.size() * NANG * 4);
            for (size_t r = 0; r < ids.size() * NANG; r++) {
                const double* m = &mats[r * NELEM];
                m4[4 * r] = m[0]; m4[4 * r + 1] = m[1]; m4[4 * r + 2] = m[10]; m4[4 * r + 3] = m[11];
            }
            HIP_TRY(upload(&W.d_mats4, m4));
        }
        HIP_TRY(upload(&W.d_matid, matid));
        W.nmat = (int)ids.size();
    }
    *out = &W;
    return 0;
}

static bool use_event_engine(const artes_grid* g) { return tv(g, T_ENGINE, 0) == 0; }

// allocate the packet pool (transport and diagnostic records) and the work lists of the
// event engine, sized for a call of n packets: a call queues at most n slots, so the pool
// holds min(default, n) slots (rounded to whole waves per sub-engine) and grows when a
// larger call arrives -- a grid that only ever runs small calls (tests, trajectory
// records) does not hold the full 8.6 GB
static void free_pool(artes_grid* g) {
    void* eptrs[] = {g->pool_mem, g->d_lists[0], g->d_lists[1], g->d_event, g->d_emit, g->d_owner};
    for (void* p : eptrs)
        if (p) hipFree(p);
    g->pool_mem = nullptr; g->d_lists[0] = g->d_lists[1] = nullptr; g->d_event = g->d_emit = nullptr; g->d_owner = nullptr;
    g->pool = Pool{};
}

static int32_t ensure_pool(artes_grid* g, uint64_t n) {
    // 128 Ki slots per CU (33.6 M on MI355X; 4.3 GB of transport records + 4.3 GB of
    // diagnostic ones): every k_trace launch ends in a tail of a few long traces
    // (~0.35 ms), so fewer, larger iterations pay it less often.  With one pool the random
    // record accesses of k_event and k_emit missed in the TLBs past ~30 M slots; split
    // over the XCDs (NSUB sub-engines) they no longer do up to 50 M (pool sweep in
    // DESIGN.md §3)
    long long Pmax = tv(g, T_POOL, (long long)g->num_cus * 131072);
    Pmax = std::max<long long>(1024, std::min<long long>(Pmax, 1LL << 26));
    long long P = std::min<long long>(Pmax, std::max<long long>((long long)std::min<uint64_t>(n, 1ULL << 26), 1024));
    auto whole = [](long long v) { return (v + 64 * NSUB - 1) / (64 * NSUB) * (64 * NSUB); };   // NSUB sub-engines of whole waves of slots
    P = whole(P);
    // a pool at least this call's size is kept unless it exceeds the pool setting (the "pool"
    // key set below an earlier call's pool reallocates: every key overrides the schedule)
    if (g->pool_mem && g->pool.P >= P && g->pool.P <= whole(Pmax)) return 0;
    free_pool(g);
    HIP_TRY(hipMalloc(&g->pool_mem, (size_t)P * (sizeof(Slot) + sizeof(SlotDiag))));
    g->pool.P = (int)P;
    g->pool.s = (Slot*)g->pool_mem;
    g->pool.d = (SlotDiag*)((char*)g->pool_mem + (size_t)P * sizeof(Slot));
    // trace lists hold up to twice the slots: a packet dropped in k_event keeps its event
    // position (a hole) and takes an emit position as well (kernel_event.hpp, Lists (L2))
    HIP_TRY(hipMalloc((void**)&g->d_lists[0], (size_t)2 * P * 4));
    HIP_TRY(hipMalloc((void**)&g->d_lists[1], (size_t)2 * P * 4));
    HIP_TRY(hipMalloc((void**)&g->d_event, (size_t)P * 4));
    HIP_TRY(hipMalloc((void**)&g->d_emit, (size_t)P * 4));
#ifdef ARTES_DEBUG
    HIP_TRY(hipMalloc((void**)&g->d_owner, (size_t)P * sizeof(int)));
#endif
    if (!g->d_counts) {
        HIP_TRY(hipMalloc((void**)&g->d_counts, CNT_FIELDS * NSUB * CPAD * sizeof(int)));
        HIP_TRY(hipMalloc((void**)&g->d_grab, 8 * NSUB * CPAD * sizeof(unsigned int)));
        HIP_TRY(hipMalloc((void**)&g->d_next, NSUB * sizeof(unsigned long long)));
        HIP_TRY(hipHostMalloc((void**)&g->h_count, 64, hipHostMallocDefault));
        HIP_TRY(hipEventCreateWithFlags(&g->ev_poll, hipEventDisableTiming));
    }
    return 0;
}

// grids are whole multiples of the sub-engine count (block b works on sub-engine b % NSUB)
static int round_sub(int blocks) { return std::max(NSUB, (blocks + NSUB - 1) / NSUB * NSUB); }

// k_trace (kernel_trace.hpp) with its face tables in LDS.  (The per-cell extinction and
// albedo in LDS as well, for grids whose table fits, measured the same as reading them from
// L2 -- cloudy 210.8 vs 211.1, hg 705 vs 707 Mpackets/s, profiles/r03/klds_ab.txt -- so they
// stay in global memory.)
// step slots per k_trace iteration of the `steps` = 4 kernel (A/B builds: ARTES_COARSE_NREP)
#ifndef ARTES_COARSE_NREP
#define ARTES_COARSE_NREP 4
#endif
// (the default kernel on fine 3D and radial-only grids: ARTES_FINE_NREP, at the top of the file)
template <bool G3D, bool OBL, int WPE, bool FLOW = false, int NREP = 8, bool GTAB = false>
static void launch_trace(artes_grid* g, int bpc, const DevGrid& G, const DevRun& R, const SubLists& L, hipStream_t stream) {
    const size_t lds = GTAB ? 0 : trace_table_bytes(G.nr, G.ntheta, G.nphi);
    const int per_cu = bpc > 0 ? bpc : blocks_per_cu(g, k_trace<G3D, OBL, WPE, FLOW, NREP, GTAB>, lds);
    g->trace_blocks = round_sub(per_cu * g->num_cus);
    g->trace_nrep = NREP;
    if (g->last_trace.empty()) {
        char b[80];
        if (GTAB) snprintf(b, sizeof(b), "k_trace<%d,%d,%d,%d,%d,1>", (int)G3D, (int)OBL, WPE, (int)FLOW, NREP);
        else snprintf(b, sizeof(b), "k_trace<%d,%d,%d,%d,%d>", (int)G3D, (int)OBL, WPE, (int)FLOW, NREP);
        g->last_trace = b;
    }
    timed(g, ARTES_K_TRACE, stream, [&] {
        hipLaunchKernelGGL((k_trace<G3D, OBL, WPE, FLOW, NREP, GTAB>), dim3(g->trace_blocks), dim3(BLOCK), lds, stream, G, R, g->pool, L);
    });
}

// k_trace variant: 3D or radial-only grid, spheroidal (oblate) or spherical planet,
// occupancy target (waves per SIMD the register budget is sized for), face tables in LDS or
// in global memory (GTAB)
// (steps: k_trace's steps per loop iteration, 8 or 4; see trace_steps)
template <bool G3D, bool GTAB>
static void launch_trace_tab(artes_grid* g, int wpe, int steps, int bpc, const DevGrid& G, const DevRun& R, const SubLists& L,
                             hipStream_t stream) {
    const bool oblate = !(G.ax2 == 1.0 && G.by2 == 1.0 && G.cz2 == 1.0 && G.a == 1.0 && G.b == 1.0);
    if (R.flow_g || R.flow_t) {   // diagnostics: one occupancy target only
        if (oblate) launch_trace<G3D, true, 4, true, 8, GTAB>(g, bpc, G, R, L, stream);
        else launch_trace<G3D, false, 4, true, 8, GTAB>(g, bpc, G, R, L, stream);
    } else if (oblate) {
        if (wpe == 3) launch_trace<G3D, true, 3, false, 8, GTAB>(g, bpc, G, R, L, stream);
        else launch_trace<G3D, true, 4, false, 8, GTAB>(g, bpc, G, R, L, stream);
    } else if (wpe == 3) {
        launch_trace<G3D, false, 3, false, 8, GTAB>(g, bpc, G, R, L, stream);
    } else if (G3D && steps == 4) {
        launch_trace<G3D, false, 4, false, ARTES_COARSE_NREP, GTAB>(g, bpc, G, R, L, stream);
    } else {
        launch_trace<G3D, false, 4, false, ARTES_FINE_NREP, GTAB>(g, bpc, G, R, L, stream);
    }
}
template <bool G3D>
static void launch_trace_any(artes_grid* g, bool gtab, int wpe, int steps, int bpc, const DevGrid& G, const DevRun& R,
                             const SubLists& L, hipStream_t stream) {
    if (gtab) launch_trace_tab<G3D, true>(g, wpe, steps, bpc, G, R, L, stream);
    else launch_trace_tab<G3D, false>(g, wpe, steps, bpc, G, R, L, stream);
}

// diagnostics (ARTES_VERBOSE) when the engine does not terminate: the transport state of
// the first packets still in the trace lists
static void dump_live(artes_grid* g, const int* cnt, int in, hipStream_t stream) {
    const int P = g->pool.P, Ps = P / NSUB;
    int n[NSUB], split[NSUB];
    if (hipMemcpy2DAsync(n, sizeof(int), cnt + cnt_at(CNT_IN0 + in, 0), CPAD * sizeof(int), sizeof(int), NSUB, hipMemcpyDeviceToHost, stream) != hipSuccess) return;
    if (hipMemcpy2DAsync(split, sizeof(int), cnt + cnt_at(CNT_SPLIT0 + in, 0), CPAD * sizeof(int), sizeof(int), NSUB, hipMemcpyDeviceToHost, stream) != hipSuccess) return;
    if (hipStreamSynchronize(stream) != hipSuccess) return;
    for (int s = 0; s < NSUB; s++) {
        fprintf(stderr, "[artes] sub-engine %d: live trace list %d entries (split %d)\n", s, n[s], split[s]);
        const int* d_list = g->d_lists[in] + (size_t)s * 2 * Ps;
        for (int j = 0; j < n[s] && j < 2; j++) {
            const int pos = j < split[s] ? j : 2 * Ps - 1 - (j - split[s]);
            int slot = -1;
            Slot r;
            SlotDiag q;
            if (hipMemcpy(&slot, d_list + pos, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess || slot < 0 || slot >= P) continue;
            if (hipMemcpy(&r, g->pool.s + slot, sizeof(Slot), hipMemcpyDeviceToHost) != hipSuccess) continue;
            if (hipMemcpy(&q, g->pool.d + slot, sizeof(SlotDiag), hipMemcpyDeviceToHost) != hipSuccess) continue;
            fprintf(stderr, "[artes] slot %d pid %llu mode %d p %.17g %.17g %.17g d %.17g %.17g %.17g ttgt %.17g cell %d face %d ncross %d nscat %d wI %.17g\n",
                    slot, q.pid, r.mode, r.px, r.py, r.pz, r.dx, r.dy, r.dz, r.ttgt, r.pcell, r.pface, r.ncross, q.nscat, r.wI);
        }
    }
}

// k_event's large block: one block per CU sharing one LDS copy of the tables;
// 768 threads = 3 waves per SIMD at <= 170 VGPRs (ARTES_EVB=1024 builds the 4-wave variant, <= 128)
#ifndef ARTES_EVB
#define ARTES_EVB 768
#endif
constexpr int EVB = ARTES_EVB;

template <bool G3D>
static int32_t run_event_engine(artes_grid* g, const DevGrid& G, const DevRun& R, bool trace, hipStream_t stream) {
    int32_t rc = ensure_pool(g, R.n);
    if (rc) return rc;
    const int P = g->pool.P, Ps = P / NSUB;
    HIP_TRY(hipMemsetAsync(g->d_counts, 0, CNT_FIELDS * NSUB * CPAD * sizeof(int), stream));
    HIP_TRY(hipMemsetAsync(g->d_grab, 0, 8 * NSUB * CPAD * sizeof(unsigned int), stream));
    HIP_TRY(hipMemsetAsync(g->d_next, 0, NSUB * sizeof(unsigned long long), stream));
    if (g->d_owner) HIP_TRY(hipMemsetAsync(g->d_owner, 0xFF, (size_t)P * sizeof(int), stream));   // tags -1: unclaimed
    int* cnt = g->d_counts;
    const int side_blocks = round_sub(g->num_cus * 8);
    // launch knobs, read once per call (tuning overrides; the defaults are the measured optima)
    const int wpe = (int)tv(g, T_WPE, 4);
    const int trace_bpc = (int)tv(g, T_TRACE_BPC, 0);   // k_trace blocks per CU (0: the occupancy limit)
    // k_trace steps per loop iteration ("Several steps per iteration"): 8 on fine
    // 3D and radial-only grids, 4 on coarse 3D grids (< 4096 cells), whose short chains leave
    // more lanes idle for the rest of an iteration (profiles/r04/ab/trace_nrep*_ab.txt);
    // tuning "steps" = 4 | 8 overrides (3D grids; the oblate, flow and wpe = 3 kernels have 8)
    const int trace_steps = (int)tv(g, T_STEPS, G.ncell < 4096 ? 4 : ARTES_FINE_NREP);
    // k_trace's face tables: in LDS up to 64 KiB (two blocks per CU at most then), beyond that
    // in global memory (GTAB kernels, L2-resident: ~2000 radial faces and more); tuning
    // "trace_gtab" = 1 forces the global tables (tests)
    const size_t ttab_bytes = trace_table_bytes(G.nr, G.ntheta, G.nphi);
    const bool gtab = ttab_bytes > 65536 || tv(g, T_TRACE_GTAB, 0) != 0;
    DevGrid GT = G;
    if (gtab) {
        if (g->ttab_cap < ttab_bytes) {
            if (g->d_ttab) hipFree(g->d_ttab);
            g->d_ttab = nullptr;
            g->ttab_cap = 0;
            HIP_TRY(hipMalloc((void**)&g->d_ttab, ttab_bytes));
            g->ttab_cap = ttab_bytes;
        }
        GT.ttab = g->d_ttab;
        hipLaunchKernelGGL(k_fill_trace_tables, dim3(1), dim3(BLOCK), 0, stream, GT);
    }
    // scattering tables in LDS for k_event when they fit next to one another (a few
    // distinct matrices: uniform and layered atmospheres); otherwise read from L2
    const size_t ev_bytes = event_table_doubles(G.nmat, G.msym != 0) * sizeof(double);
    const bool ev_lds = tv(g, T_EVENT_LDS, 1) != 0 && ev_bytes <= 65536;
    // planes 0-8 of the detector accumulated per k_event block in LDS when they fit
    // (the I-only count plane 9 of the rare thermal / surface peels goes straight to HBM):
    // with the scattering tables, 76.7 KB at 25x25 pixels, so two blocks share a CU
    const size_t det_bytes = 9 * (size_t)R.nx * R.ny * sizeof(double);
    // one-pixel detector (spectrum / phase): per-lane register sums reduced over the wave
    // (k_event PIX1) instead of same-address atomics; tuning "pix1" = 0 turns it off
    const bool pix1 = tv(g, T_PIX1, 1) != 0 && R.nx == 1 && R.ny == 1;
    // k_event's block with both the tables and the detector in LDS: EVB threads, one block
    // (12 waves, 3 per SIMD at <= 170 VGPRs) per CU sharing one LDS copy, instead of two
    // 256-thread blocks (2 waves per SIMD, LDS-bound): k_event -7 % on ray3d / hg / iso
    // (tuning "event_block" = 256 for the old shape)
    const int ev_block = tv(g, T_EVENT_BLOCK, EVB) == 256 ? 256 : EVB;
    // matrices too many for LDS: their cumulative tables alone in LDS (k_event LDS_C) when
    // they fit beside the detector or the one-pixel lane slots in one EVB-thread block per
    // CU; tuning "event_ldsc" = 0 turns it off
    const size_t cum_bytes = event_cum_doubles(G.nmat) * sizeof(double);
    const bool ev_ldsc_ok = !ev_lds && ev_block == EVB && tv(g, T_EVENT_LDSC, 1) != 0;
    const bool det_lds = !pix1 && tv(g, T_DET_LDS, 1) != 0 && (ev_lds ? ev_bytes : 0) + det_bytes <= 98304;
    const size_t lds_cap = 160 * 1024 - 4096;   // (a margin for static LDS)
    const bool ev_ldsc = ev_ldsc_ok && cum_bytes + (pix1 ? pix1_slot_bytes(EVB) : det_lds ? det_bytes : 0) <= lds_cap;
    const size_t tab_bytes = ev_lds ? ev_bytes : (ev_ldsc ? cum_bytes : 0);
    int ev_blocks = side_blocks;
    if (det_lds) {
        const size_t b = tab_bytes + det_bytes;
        int per_cu = ev_block == EVB ? (ev_lds ? blocks_per_cu(g, k_event<true, true, false, EVB>, b, EVB)
                                               : ev_ldsc ? blocks_per_cu(g, k_event<false, true, false, EVB, true>, b, EVB)
                                                         : blocks_per_cu(g, k_event<false, true, false, EVB>, b, EVB))
                                     : (ev_lds ? blocks_per_cu(g, k_event<true, true>, b) : blocks_per_cu(g, k_event<false, true>, b));
        per_cu = (int)tv(g, T_EVENT_BPC, per_cu);
        ev_blocks = round_sub(per_cu * g->num_cus);
    }
    // the one-pixel kernel in EVB-thread blocks too: the launch bound holds it to 3 waves per
    // SIMD (<= 168 VGPRs; 211-219 at 256 threads, i.e. 2 waves)
    const bool pix1_big = pix1 && ev_block == EVB;
    const size_t p1_bytes = tab_bytes + pix1_slot_bytes(pix1_big ? EVB : BLOCK);
    if (pix1_big) {
        const int per_cu = ev_lds ? blocks_per_cu(g, k_event<true, false, true, EVB>, p1_bytes, EVB)
                                  : ev_ldsc ? blocks_per_cu(g, k_event<false, false, true, EVB, true>, p1_bytes, EVB)
                                            : blocks_per_cu(g, k_event<false, false, true, EVB>, p1_bytes, EVB);
        ev_blocks = round_sub(per_cu * g->num_cus);
    }
    // the global-detector kernel with LDS_C: one EVB-thread block per CU as well
    const bool glob_ldsc = ev_ldsc && !pix1 && !det_lds;
    if (glob_ldsc) ev_blocks = round_sub(blocks_per_cu(g, k_event<false, false, false, EVB, true>, cum_bytes, EVB) * g->num_cus);
    // the packet ids of the call split into NSUB contiguous ranges, one per sub-engine
    const uint64_t chunk = (R.n + NSUB - 1) / NSUB;
    uint64_t sub_first[NSUB], sub_n[NSUB];
    for (int s = 0; s < NSUB; s++) {
        const uint64_t lo = std::min<uint64_t>(R.n, (uint64_t)s * chunk), hi = std::min<uint64_t>(R.n, lo + chunk);
        sub_first[s] = R.first + lo;
        sub_n[s] = hi - lo;
    }
    auto lists = [&](int in) {
        SubLists SL;
        for (int s = 0; s < NSUB; s++) {
            Lists& L = SL.l[s];
            const size_t o = (size_t)s * Ps, ot = (size_t)s * 2 * Ps;
            L.trace_in = g->d_lists[in] + ot; L.trace_in_n = cnt + cnt_at(CNT_IN0 + in, s);
            L.trace_in_split = cnt + cnt_at(CNT_SPLIT0 + in, s);
            L.trace_out = g->d_lists[1 - in] + ot; L.trace_out_n = cnt + cnt_at(CNT_IN0 + 1 - in, s);
            L.event = g->d_event + o; L.event_n = cnt + cnt_at(CNT_EVENT, s);
            L.emit = g->d_emit + o; L.emit_n = cnt + cnt_at(CNT_EMIT, s);
            L.grab = g->d_grab + grab_at(s, 0); L.next_pkt = g->d_next + s;
            L.dbg_owner = g->d_owner; L.dbg_iter = cnt + cnt_at(CNT_DBG, s);
            L.P = 2 * Ps; L.first = sub_first[s]; L.n = sub_n[s];
        }
        return SL;
    };
    const size_t em_lds = G3D ? emit_table_doubles(G.ntheta, G.nphi) * sizeof(double) : 0;
    auto launch_emit = [&](const SubLists& L) {
        const bool star = R.photon_source != 2;
        if (trace) hipLaunchKernelGGL((k_emit<G3D, true>), dim3(side_blocks), dim3(BLOCK), em_lds, stream, G, R, g->pool, L);
        else if (star) hipLaunchKernelGGL((k_emit<G3D, false, true>), dim3(side_blocks), dim3(BLOCK), em_lds, stream, G, R, g->pool, L);
        else hipLaunchKernelGGL((k_emit<G3D, false>), dim3(side_blocks), dim3(BLOCK), em_lds, stream, G, R, g->pool, L);
    };
    SubUse use;
    for (int s = 0; s < NSUB; s++) use.u[s] = (int)std::min<uint64_t>((uint64_t)Ps, std::max<uint64_t>(sub_n[s], 1));
    timed(g, ARTES_K_AUX, stream, [&] {
        hipLaunchKernelGGL(k_init, dim3(((size_t)P + 255) / 256), dim3(256), 0, stream, g->pool, g->d_emit, cnt + cnt_at(CNT_EMIT, 0), Ps, use);
    });
    // pre-iteration: fill the pool; emitted packets go to trace list 0
    {
        SubLists L = lists(1);   // trace_out = list 0
        timed(g, ARTES_K_EMIT, stream, [&] { launch_emit(L); });
        timed(g, ARTES_K_AUX, stream, [&] {
            hipLaunchKernelGGL(k_rotate, dim3(NSUB), dim3(64), 0, stream, cnt, 1, g->d_grab, g->d_next, R.emit_first, 2 * Ps, R.err);
        });
    }
    // The k_event instantiation of this call (fixed for the call; its name is reported by
    // artes_last_launch): tables in LDS (LDS_T) or only their cumulative part (LDS_C), the
    // detector in LDS (LDS_D) or per-lane one-pixel sums (PIX1), 768- or 256-thread blocks.
    // tests/test_gpu_event_variants.py forces every branch and checks it against the oracle.
    int ev_v = 13;
    if (pix1_big && ev_lds) ev_v = 1;
    else if (pix1_big && ev_ldsc) ev_v = 2;
    else if (det_lds && ev_ldsc) ev_v = 3;
    else if (glob_ldsc) ev_v = 4;
    else if (pix1_big) ev_v = 5;
    else if (pix1 && ev_lds) ev_v = 6;
    else if (pix1) ev_v = 7;
    else if (ev_lds && det_lds && ev_block == EVB) ev_v = 8;
    else if (ev_lds && det_lds) ev_v = 9;
    else if (ev_lds) ev_v = 10;
    else if (det_lds && ev_block == EVB) ev_v = 11;
    else if (det_lds) ev_v = 12;
    // the call's tables too many for LDS padded but not unpadded (the global layout: the cloudy
    // calls' 9 matrices per wavelength, 104 KB against 130 KB padded) beside the one-pixel lane
    // slots or the LDS detector: k_event TPAD = false instead of the cumulative tables alone
    // (tuning "event_ldsu" = 0 turns it off; profiles/r06/ab/event_tables_unpadded_ab.txt)
    const size_t evu_bytes = event_table_doubles_unpadded(G.nmat, G.msym != 0) * sizeof(double);
    if (!ev_lds && ev_block == EVB && tv(g, T_EVENT_LDS, 1) != 0 && tv(g, T_EVENT_LDSU, 1) != 0) {
        if (pix1_big && evu_bytes + pix1_slot_bytes(EVB) <= lds_cap) {
            ev_v = 17;
            ev_blocks = round_sub(blocks_per_cu(g, k_event<true, false, true, EVB, false, 0, false>,
                                                evu_bytes + pix1_slot_bytes(EVB), EVB) * g->num_cus);
        } else if (det_lds && evu_bytes + det_bytes <= lds_cap) {
            ev_v = 18;
            ev_blocks = round_sub((int)tv(g, T_EVENT_BPC, blocks_per_cu(g, k_event<true, true, false, EVB, false, 0, false>,
                                                                         evu_bytes + det_bytes, EVB)) * g->num_cus);
        }
    }
    // det_ordered: the fixed-point detector (k_event ORD), EVB-thread blocks, the tables in LDS as
    // far as they fit alone
    // (the block's integer sums in LDS when they fit beside the tables -- 160 B per pixel: 25 x 25
    // imaging 100 KB, a one-pixel detector 160 B -- else added to the HBM copy at once)
    const size_t fixl_bytes = 20 * (size_t)R.nx * R.ny * sizeof(unsigned long long);
    const bool ord_ldsc = cum_bytes <= lds_cap && tv(g, T_EVENT_LDSC, 1) != 0;
    if (R.fix) {
        if (ev_lds && ev_bytes + fixl_bytes <= lds_cap) ev_v = 14;
        else if (ord_ldsc && cum_bytes + fixl_bytes <= lds_cap) ev_v = 15;
        else if (fixl_bytes <= lds_cap) ev_v = 16;
        else ev_v = ord_ldsc ? 19 : 20;
        ev_blocks = round_sub((ev_v == 14 ? blocks_per_cu(g, k_event<true, false, false, EVB, false, 2>, ev_bytes + fixl_bytes, EVB)
                               : ev_v == 15 ? blocks_per_cu(g, k_event<false, false, false, EVB, true, 2>, cum_bytes + fixl_bytes, EVB)
                               : ev_v == 16 ? blocks_per_cu(g, k_event<false, false, false, EVB, false, 2>, fixl_bytes, EVB)
                               : ev_v == 19 ? blocks_per_cu(g, k_event<false, false, false, EVB, true, 1>, cum_bytes, EVB)
                                            : blocks_per_cu(g, k_event<false, false, false, EVB, false, 1>, 0, EVB)) * g->num_cus);
    }
    static const struct { int lt, ld, p1, big, lc, ord, tpad; } EVV[21] = {
        {0, 0, 0, 0, 0, 0, 1}, {1, 0, 1, 1, 0, 0, 1}, {0, 0, 1, 1, 1, 0, 1}, {0, 1, 0, 1, 1, 0, 1}, {0, 0, 0, 1, 1, 0, 1},
        {0, 0, 1, 1, 0, 0, 1}, {1, 0, 1, 0, 0, 0, 1}, {0, 0, 1, 0, 0, 0, 1}, {1, 1, 0, 1, 0, 0, 1}, {1, 1, 0, 0, 0, 0, 1},
        {1, 0, 0, 0, 0, 0, 1}, {0, 1, 0, 1, 0, 0, 1}, {0, 1, 0, 0, 0, 0, 1}, {0, 0, 0, 0, 0, 0, 1}, {1, 0, 0, 1, 0, 2, 1},
        {0, 0, 0, 1, 1, 2, 1}, {0, 0, 0, 1, 0, 2, 1}, {1, 0, 1, 1, 0, 0, 0}, {1, 1, 0, 1, 0, 0, 0}, {0, 0, 0, 1, 1, 1, 1},
        {0, 0, 0, 1, 0, 1, 1}};
    {
        // (the template arguments LDS_T, LDS_D, PIX1, block, LDS_C, then ORD and TPAD where they are not the defaults)
        const auto& V = EVV[ev_v];
        char b[96];
        if (!V.tpad) snprintf(b, sizeof(b), "k_event<%d,%d,%d,%d,%d,%d,0>", V.lt, V.ld, V.p1, V.big ? EVB : BLOCK, V.lc, V.ord);
        else if (V.ord) snprintf(b, sizeof(b), "k_event<%d,%d,%d,%d,%d,%d>", V.lt, V.ld, V.p1, V.big ? EVB : BLOCK, V.lc, V.ord);
        else snprintf(b, sizeof(b), "k_event<%d,%d,%d,%d,%d>", V.lt, V.ld, V.p1, V.big ? EVB : BLOCK, V.lc);
        g->last_event = b;
    }
    auto launch_event = [&](const SubLists& L) {
        switch (ev_v) {
        case 1: hipLaunchKernelGGL((k_event<true, false, true, EVB>), dim3(ev_blocks), dim3(EVB), p1_bytes, stream, G, R, g->pool, L); break;
        case 2: hipLaunchKernelGGL((k_event<false, false, true, EVB, true>), dim3(ev_blocks), dim3(EVB), p1_bytes, stream, G, R, g->pool, L); break;
        case 3: hipLaunchKernelGGL((k_event<false, true, false, EVB, true>), dim3(ev_blocks), dim3(EVB), cum_bytes + det_bytes, stream, G, R, g->pool, L); break;
        case 4: hipLaunchKernelGGL((k_event<false, false, false, EVB, true>), dim3(ev_blocks), dim3(EVB), cum_bytes, stream, G, R, g->pool, L); break;
        case 5: hipLaunchKernelGGL((k_event<false, false, true, EVB>), dim3(ev_blocks), dim3(EVB), p1_bytes, stream, G, R, g->pool, L); break;
        case 6: hipLaunchKernelGGL((k_event<true, false, true>), dim3(side_blocks), dim3(BLOCK), p1_bytes, stream, G, R, g->pool, L); break;
        case 7: hipLaunchKernelGGL((k_event<false, false, true>), dim3(side_blocks), dim3(BLOCK), p1_bytes, stream, G, R, g->pool, L); break;
        case 8: hipLaunchKernelGGL((k_event<true, true, false, EVB>), dim3(ev_blocks), dim3(EVB), ev_bytes + det_bytes, stream, G, R, g->pool, L); break;
        case 9: hipLaunchKernelGGL((k_event<true, true>), dim3(ev_blocks), dim3(BLOCK), ev_bytes + det_bytes, stream, G, R, g->pool, L); break;
        case 10: hipLaunchKernelGGL((k_event<true, false>), dim3(side_blocks), dim3(BLOCK), ev_bytes, stream, G, R, g->pool, L); break;
        case 11: hipLaunchKernelGGL((k_event<false, true, false, EVB>), dim3(ev_blocks), dim3(EVB), det_bytes, stream, G, R, g->pool, L); break;
        case 12: hipLaunchKernelGGL((k_event<false, true>), dim3(ev_blocks), dim3(BLOCK), det_bytes, stream, G, R, g->pool, L); break;
        case 14: hipLaunchKernelGGL((k_event<true, false, false, EVB, false, 2>), dim3(ev_blocks), dim3(EVB), ev_bytes + fixl_bytes, stream, G, R, g->pool, L); break;
        case 15: hipLaunchKernelGGL((k_event<false, false, false, EVB, true, 2>), dim3(ev_blocks), dim3(EVB), cum_bytes + fixl_bytes, stream, G, R, g->pool, L); break;
        case 16: hipLaunchKernelGGL((k_event<false, false, false, EVB, false, 2>), dim3(ev_blocks), dim3(EVB), fixl_bytes, stream, G, R, g->pool, L); break;
        case 17: hipLaunchKernelGGL((k_event<true, false, true, EVB, false, 0, false>), dim3(ev_blocks), dim3(EVB), evu_bytes + pix1_slot_bytes(EVB), stream, G, R, g->pool, L); break;
        case 18: hipLaunchKernelGGL((k_event<true, true, false, EVB, false, 0, false>), dim3(ev_blocks), dim3(EVB), evu_bytes + det_bytes, stream, G, R, g->pool, L); break;
        case 19: hipLaunchKernelGGL((k_event<false, false, false, EVB, true, 1>), dim3(ev_blocks), dim3(EVB), cum_bytes, stream, G, R, g->pool, L); break;
        case 20: hipLaunchKernelGGL((k_event<false, false, false, EVB, false, 1>), dim3(ev_blocks), dim3(EVB), 0, stream, G, R, g->pool, L); break;
        default: hipLaunchKernelGGL((k_event<false, false>), dim3(side_blocks), dim3(BLOCK), 0, stream, G, R, g->pool, L); break;
        }
    };
    HIP_TRY(hipGetLastError());
    int in = 0;
    long long it = 0;
    const long long max_it = tv(g, T_MAX_IT, 2000000LL);
    g->prof_loop = true;
    g->prof_chain = false;
    struct LoopEnd { artes_grid* g; ~LoopEnd() { g->prof_loop = false; g->prof_chain = false; } } loop_end{g};
    for (;;) {
        SubLists L = lists(in);
        launch_trace_any<G3D>(g, gtab, wpe, trace_steps, trace_bpc, GT, R, L, stream);
        timed(g, ARTES_K_EVENT, stream, [&] { launch_event(L); });
        timed(g, ARTES_K_EMIT, stream, [&] { launch_emit(L); });
        timed(g, ARTES_K_AUX, stream, [&] {
            hipLaunchKernelGGL(k_rotate, dim3(NSUB), dim3(64), 0, stream, cnt, in, g->d_grab, g->d_next, R.emit_first, 2 * Ps, R.err);
        });
        in = 1 - in;
        it++;
        if ((it & 7) == 0 || it < 4) {   // poll the live-packet count (trace list of the next iteration)
            HIP_TRY(hipGetLastError());
            // (and the watchdog counter: a schedule bug fails the run at once instead of
            // every launch spinning to the watchdog)
            unsigned long long* h_wd = (unsigned long long*)(g->h_count + NSUB);
            HIP_TRY(hipMemcpy2DAsync(g->h_count, sizeof(int), cnt + cnt_at(CNT_IN0 + in, 0), CPAD * sizeof(int), sizeof(int), NSUB, hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipMemcpyAsync(h_wd, R.err + ARTES_ERR_WATCHDOG, sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipEventRecord(g->ev_poll, stream));
            g->prof_chain = false;   // (the copies sit between this launch and the next)
            HIP_TRY(hipEventSynchronize(g->ev_poll));
            if (*h_wd) return fail(-5, "transport kernel watchdog fired: schedule bug, results invalid");
            long long live = 0;
            for (int s = 0; s < NSUB; s++) live += g->h_count[s];
            if (live == 0) break;
        }
        if (it > max_it) {
            if (tv(g, T_VERBOSE, 0)) dump_live(g, cnt, in, stream);
            return fail(-5, "event engine did not terminate");
        }
    }
    g->last_iterations = it;
    if (tv(g, T_VERBOSE, 0))
        fprintf(stderr, "[artes] event engine: pool %d, %lld iterations, trace blocks %d (%d steps per iteration), event blocks %d (LDS tables %d, cumulative tables %d, detector %d, 1-pixel %d, matrices %d)\n",
                P, it, g->trace_blocks, g->trace_nrep, ev_blocks, (int)ev_lds, (int)ev_ldsc, (int)det_lds, (int)pix1, G.nmat);
    return 0;
}

extern "C" {

static int32_t launch(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                      double* det_out, double* tot_out, unsigned long long* cnt_out, unsigned long long* err_out,
                      double* rec, hipStream_t stream, double* flow_g = nullptr, double* flow_t = nullptr) {
    const HostTables& T = g->T;
    if (!p) return fail(-22, "null params");
    g->last_trace.clear();
    g->last_event.clear();
    g->last_engine = 0;
    if (p->photon_source != 1 && p->photon_source != 2) return fail(-22, "photon_source must be 1 (star) or 2 (planet)");
    if (!use_event_engine(g) && (p->photon_source != 1 || p->surface_albedo > 0.0 || flow_g || flow_t))
        return fail(-38, "the persistent engine supports the star source without surface reflection or flow output only");
    if (p->wl_index < 0 || p->wl_index >= T.nwav) return fail(-22, "wl_index out of range");
    if (p->nx < 1 || p->ny < 1 || (size_t)p->nx * p->ny > (1u << 26)) return fail(-22, "bad detector size");
    HIP_TRY(hipSetDevice(g->device));
    const size_t plane = (size_t)p->nx * p->ny;
    const size_t stride = (16 * plane + 31) & ~(size_t)31;   // (copies on 256-byte lines of their own)
    const int ncopy = det_copies(stride);
    if (g->copies_cap < stride * ncopy) {
        if (g->d_copies) hipFree(g->d_copies);
        g->d_copies = nullptr;
        HIP_TRY(hipMalloc((void**)&g->d_copies, stride * ncopy * sizeof(double)));
        g->copies_cap = stride * ncopy;
    }
    HIP_TRY(hipMemsetAsync(g->d_copies, 0, stride * ncopy * sizeof(double), stream));
    // det_ordered: the fixed-point copies of planes 0-9, one per CU (a k_event block's copy is its
    // index modulo nfix) within 256 MiB
    const bool det_ordered = tv(g, T_DET_ORDERED, 0) != 0;
    if (det_ordered && !use_event_engine(g)) return fail(-38, "det_ordered: the event engine only");
    const size_t fix_stride = 20 * plane;
    int nfix = 0;
    if (det_ordered) {
        nfix = (int)std::max<size_t>(1, std::min<size_t>((size_t)g->num_cus, ((size_t)256 << 20) / (fix_stride * 8)));
        if (g->fix_cap < fix_stride * nfix) {
            if (g->d_fix) hipFree(g->d_fix);
            g->d_fix = nullptr;
            g->fix_cap = 0;
            HIP_TRY(hipMalloc((void**)&g->d_fix, fix_stride * nfix * sizeof(unsigned long long)));
            g->fix_cap = fix_stride * nfix;
        }
        HIP_TRY(hipMemsetAsync(g->d_fix, 0, fix_stride * nfix * sizeof(unsigned long long), stream));
    }

    DevGrid G;
    G.nr = T.nr; G.ntheta = T.ntheta; G.nphi = T.nphi; G.ncell = T.ncell; G.nmat = T.nmat;
    G.cell_depth = p->cell_depth >= 0 ? p->cell_depth : T.cell_depth[p->wl_index];
    G.rfr = g->d_rfront; G.tcos = g->d_tcos;
    G.ttab = nullptr;
    G.ox = T.oblate_x; G.oy = T.oblate_y; G.oz = T.oblate_z;
    G.th_cdf = nullptr; G.th_weight = nullptr; G.th_ncdf = 0; G.th_cd0 = 0; G.th_total = 0.0;
    if (p->photon_source == 2) {   // thermal tables of this wavelength (ARTES.f90:2359-2453)
        ThermalTables X;
        try {
            X = build_thermal(T, p->wl_index, p->thermal_weight != 0, p->ring != 0);
        } catch (const std::exception& e) {
            return fail(-22, e.what());
        }
        if (!(X.total > 0.0)) return fail(-22, "planet source: the atmosphere emits nothing at this wavelength");
        const size_t need = std::max(X.cdf.size(), X.weight.size());
        if (g->th_cap < need) {
            if (g->d_th_cdf) hipFree(g->d_th_cdf);
            if (g->d_th_weight) hipFree(g->d_th_weight);
            g->d_th_cdf = g->d_th_weight = nullptr;
            HIP_TRY(hipMalloc((void**)&g->d_th_cdf, need * sizeof(double)));
            HIP_TRY(hipMalloc((void**)&g->d_th_weight, need * sizeof(double)));
            g->th_cap = need;
        }
        HIP_TRY(hipMemcpyAsync(g->d_th_cdf, X.cdf.data(), X.cdf.size() * sizeof(double), hipMemcpyHostToDevice, stream));
        HIP_TRY(hipMemcpyAsync(g->d_th_weight, X.weight.data(), X.weight.size() * sizeof(double), hipMemcpyHostToDevice, stream));
        HIP_TRY(hipStreamSynchronize(stream));   // the host vectors go out of scope
        G.th_cdf = g->d_th_cdf; G.th_weight = g->d_th_weight;
        G.th_ncdf = (int)X.cdf.size(); G.th_cd0 = X.cell_depth; G.th_total = X.total;
        if (p->cell_depth < 0) G.cell_depth = X.cell_depth;
    }
    G.ax2 = 1.0 / (T.oblate_x * T.oblate_x); G.by2 = 1.0 / (T.oblate_y * T.oblate_y); G.cz2 = 1.0 / (T.oblate_z * T.oblate_z);
    G.a = 1.0 / T.oblate_x; G.b = 1.0 / T.oblate_y;
    G.rtop = T.rfront[T.nr];
    G.rf2 = g->d_rf2; G.thetaf = g->d_thetaf; G.tan2 = g->d_tan2; G.tplane = g->d_tplane;
    G.phif = g->d_phif; G.phis = g->d_phis; G.phic = g->d_phic;
    G.kappa = g->d_kappa + (size_t)p->wl_index * T.ncell;
    G.albedo = g->d_albedo + (size_t)p->wl_index * T.ncell;
    // k_trace's per-cell table: (kappa, gamma), gamma the scattering-loop head's weight
    // albedo / (1 - fstop) where 0 < albedo < 1, else 1 (ARTES.f90:801-805) -- the reference's
    // division, done once per cell on the host instead of per interaction on the device
    // (a multiply by 1 where the reference skips it: the same weight bit for bit); rebuilt
    // when a call brings another fstop
    if (g->ka_fstop != p->fstop) {
        std::vector<double> ka(2 * T.kappa.size());
        const double om = 1.0 - p->fstop;
        for (size_t i = 0; i < T.kappa.size(); i++) {
            const double a = T.albedo[i];
            ka[2 * i] = T.kappa[i];
            ka[2 * i + 1] = (a < 1.0 && a > 0.0) ? a / om : 1.0;
        }
        HIP_TRY(hipStreamSynchronize(stream));   // (no earlier call on this stream still reads the old table)
        HIP_TRY(hipMemcpyAsync(g->d_ka, ka.data(), ka.size() * sizeof(double), hipMemcpyHostToDevice, stream));
        HIP_TRY(hipStreamSynchronize(stream));   // (the host vector goes out of scope)
        g->ka_fstop = p->fstop;
    }
    G.ka = g->d_ka + 2 * (size_t)p->wl_index * T.ncell;
    {
        artes_grid::WlSet* W = nullptr;
        const int32_t rc = wl_set(g, p->wl_index, &W);
        if (rc) return rc;
        G.nmat = W->nmat; G.matid = W->d_matid; G.cums = W->d_cums;
        // (the persistent engine reads the 16-element form; tuning "msym" = 0, read per call, too)
        G.msym = (W->d_mats4 && use_event_engine(g) && tv(g, T_MSYM, 1) != 0) ? 1 : 0;
        G.mats = G.msym ? W->d_mats4 : W->d_mats;
    }
    G.sc2 = g->d_sc2; G.ss2 = g->d_ss2;

    DevRun R;
    R.first = first; R.n = n; R.seed = seed;
    R.nx = p->nx; R.ny = p->ny; R.photon_scattering = p->photon_scattering; R.phase_far = p->phase_far;
    R.photon_source = p->photon_source; R.photon_emission = p->photon_emission; R.photon_bias = p->photon_bias;
    R.moments = p->packet_moments != 0 || rec != nullptr;
    R.stellar_direction = p->stellar_direction;
    R.defer = (int)tv(g, T_DEFER, 16);
    // refill a wave once this many of its lanes are idle (re-swept after the batched
    // interactions: 16 on 3D grids, 20 on radial-only ones)
    const bool grid3d = (T.ntheta > 1 || T.nphi > 1);
    // (coarse 3D grids -- the cloudy atmospheres of configs[3], ~600 cells -- have short traces
    // and refill best at 32: cloudy phase +2.7 %, spectrum +4 %, profiles/r03/cloudy_ldsc_refill.txt)
    // (round 4, with the trace-relative radial family: radial-only grids 28 -- hg +2 %, iso +14 %
    // against 20 -- and coarse 3D grids 28 -- the cloudy calls +1.5 % against 32; fine 3D grids
    // stay at 16; profiles/r04/ab/refill_after_trel.txt)
    // (with 4 steps per k_trace iteration on coarse 3D grids: 20 there, with theta batches of 8 --
    // the cloudy calls +1.8 %, two runs; profiles/r04/ab/cloudy_refill_gbatch_theta2.txt)
    // (round 5, with the counters on lines of their own, the takes are cheaper: 16 on all 3D
    // grids -- the cloudy calls +0.4 % against 20 -- and 20 on radial-only ones -- hg +0.5 %,
    // iso +0.2 % against 28; profiles/r05/ab/pad_refill.txt)
    R.refill = (int)tv(g, T_REFILL, grid3d ? 16 : 20);
    // ended chains' list appends at the wave's next refill (kernel_trace.hpp `append`): ray3d
    // +3.7 %, hg +5.1 %, iso +2.7 %, the cloudy configs[3] calls +3.4-3.8 % (3e8 / 1e8 packets,
    // profiles/r03/late_append_ab.txt)
    R.late_append = (int)tv(g, T_LATE_APPEND, 1);
    R.emit_first = (int)tv(g, T_EMIT_FIRST, grid3d ? 0 : 1);
    R.backward = (int)tv(g, T_BACKWARD, 1);
    // lanes that park for the batched forced first interaction (kernel_trace.hpp): run the
    // block once this many wait, or once fewer than batch_min lanes still step (2 since the
    // common set-up block: ray3d +0.5 %, cloudy +0.3 %, hg / iso +0.2 %; 1 before,
    // profiles/r05/ab/knobs_batch_hbatch.txt)
    R.batch = (int)tv(g, T_BATCH, 2);
    // (>= 1: a wave whose stepping lanes all wait for a batch must run it)
    R.batch_min = (int)tv(g, T_BATCH_MIN, 16);
    // lanes whose propagation reached its interaction point park the same way: the
    // interaction block (roulette, albedo weight) runs once this many wait: 4 (3D grids had 6
    // while the block also set up the peel-off traces, which the common set-up block does
    // now: ray3d +0.3 % at 4, cloudy the same; profiles/r05/ab/knobs_batch_hbatch.txt)
    R.hbatch = (int)tv(g, T_HBATCH, 4);
    // trace-relative kernels: a lane whose nearest entry is a theta / phi bound waits until
    // this many lanes of the wave need that evaluation (or few lanes still step), so the
    // wave runs the theta / phi form in fewer slots.  Only the 4-step kernel
    // (coarse grids, or steps = 4) batches: 8 there (2: cloudy -2.3 %); the 8-step kernel
    // evaluates at once since the radial-form slots (waiting for 4 measured 3.5 % slower on
    // ray3d; profiles/r05/ab/knobs_gbatch*.txt)
    R.gbatch = (int)tv(g, T_GBATCH, 8);
    // the least list entries a dynamic grab of k_trace asks for (the wave keeps the rest for
    // its next refills; kernel_event.hpp, wave_take): 64 since the shard cursors have lines of
    // their own (cloudy +0.8 %, the rest the same as 128; profiles/r05/ab/pad_knobs.txt)
    R.dgrab = (int)tv(g, T_DGRAB, 64);
    // statically dealt share of the trace list, in 1/64 (the rest is grabbed dynamically):
    // 32 on 3D grids, 24 on radial-only ones since the dynamic grabs ask for 128 entries
    // (48 / 40 before: each grab was an atomic round trip; profiles/r04/ab/dyn_grab_sweep2_static.txt)
    R.static_q64 = (int)tv(g, T_STATIC, grid3d ? 32 : 24);
    R.det0 = sin(p->det_theta) * cos(p->det_phi);   // spherical_cartesian (ARTES.f90:495)
    R.det1 = sin(p->det_theta) * sin(p->det_phi);
    R.det2 = cos(p->det_theta);
    R.sdt = sin(p->det_theta); R.cdt = cos(p->det_theta); R.sdp = sin(p->det_phi); R.cdp = cos(p->det_phi);
    R.det_phi = atan2(R.det1, R.det0);
    if (R.det_phi < 0.0) R.det_phi += 2.0 * M_PI;
    if (R.det_phi > 2.0 * M_PI) R.det_phi -= 2.0 * M_PI;
    R.cdphi = cos(R.det_phi); R.sdphi = sin(R.det_phi);
    R.x_max = p->x_max; R.y_max = p->y_max; R.fstop = p->fstop; R.pmin = p->photon_minimum;
    R.surface_albedo = p->surface_albedo; R.theta_star = p->theta_star; R.phi_star = p->phi_star;
    R.det = g->d_copies; R.det_stride = stride; R.ncopy = ncopy;
    R.fix = det_ordered ? g->d_fix : nullptr; R.fix_stride = fix_stride; R.nfix = std::max(nfix, 1);
    R.tot2 = g->d_tot_part; R.cnt = g->d_cnt_part; R.err = err_out; R.rec = rec;
    HIP_TRY(hipMemsetAsync(g->d_cnt_part, 0, CNT_COPIES * CNT_STRIDE * sizeof(unsigned long long), stream));
    HIP_TRY(hipMemsetAsync(g->d_tot_part, 0, CNT_COPIES * CNT_STRIDE * sizeof(double), stream));
    R.flow_g = flow_g; R.flow_t = flow_t;

    const bool g3d = (T.ntheta > 1 || T.nphi > 1);
    HIP_TRY(hipEventRecord(g->ev0, stream));
    if (n > 0 && use_event_engine(g)) {
        if (T.nr >= 4096 || T.ntheta >= 1024 || T.nphi >= 1024)
            return fail(-22, "event engine packs cells into 12/10/10 bits: nr < 4096, ntheta < 1024, nphi < 1024");
        if ((long long)T.ncell >= (1LL << 28))
            return fail(-22, "event engine addresses the per-cell table with 32-bit byte offsets: ncell < 2^28");
        g->last_engine = 1;
        int32_t rc = g3d ? run_event_engine<true>(g, G, R, rec != nullptr, stream)
                         : run_event_engine<false>(g, G, R, rec != nullptr, stream);
        if (rc) {
            // the counters and totals of what did run still reach the caller (a failed run's
            // error codes are already in err_out): fold the partials before reporting the failure
            hipLaunchKernelGGL(sum_counters, dim3(1), dim3(64), 0, stream, (const unsigned long long*)g->d_cnt_part,
                               cnt_out, (const double*)g->d_tot_part, tot_out);
            return rc;
        }
    } else if (n > 0) {
        uint64_t want = (n + BLOCK - 1) / BLOCK;
        int blocks = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)g->max_blocks));
        g->last_engine = 2;
        timed(g, ARTES_K_PERSISTENT, stream, [&] {
            if (rec) {
                if (g3d) hipLaunchKernelGGL((transport_kernel<true, true>), dim3(blocks), dim3(BLOCK), 0, stream, G, R);
                else hipLaunchKernelGGL((transport_kernel<false, true>), dim3(blocks), dim3(BLOCK), 0, stream, G, R);
            } else {
                if (g3d) hipLaunchKernelGGL((transport_kernel<true, false>), dim3(blocks), dim3(BLOCK), 0, stream, G, R);
                else hipLaunchKernelGGL((transport_kernel<false, false>), dim3(blocks), dim3(BLOCK), 0, stream, G, R);
            }
        });
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipEventRecord(g->ev1, stream));
    g->timed = true;
    const int rb = (int)((16 * plane + 255) / 256);
    timed(g, ARTES_K_AUX, stream, [&] {
        if (det_ordered)
            hipLaunchKernelGGL(reduce_fixed, dim3((unsigned)((10 * plane + 255) / 256)), dim3(256), 0, stream,
                               (const unsigned long long*)g->d_fix, fix_stride, nfix, plane, g->d_copies);
        hipLaunchKernelGGL(reduce_detector, dim3(rb), dim3(256), 0, stream, (const double*)g->d_copies, stride, ncopy, plane, det_out);
        hipLaunchKernelGGL(sum_counters, dim3(1), dim3(64), 0, stream, (const unsigned long long*)g->d_cnt_part, cnt_out,
                           (const double*)g->d_tot_part, tot_out);
    });
    HIP_TRY(hipGetLastError());
    return 0;
}

int32_t artes_run_device(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                         double* det_dev, double* tot_dev, uint64_t* cnt_dev, uint64_t* err_dev, void* stream) {
    if (!g || !det_dev) return fail(-22, "null argument");
    HIP_TRY(hipSetDevice(g->device));
    hipStream_t s = (hipStream_t)stream;
    if (!tot_dev) { HIP_TRY(hipMemsetAsync(g->d_tot, 0, 6 * sizeof(double), s)); }
    if (!cnt_dev) { HIP_TRY(hipMemsetAsync(g->d_cnt, 0, ARTES_NUM_COUNTERS * 8, s)); }
    if (!err_dev) { HIP_TRY(hipMemsetAsync(g->d_err, 0, ARTES_NUM_ERR * 8, s)); }
    return launch(g, p, first, n, seed, det_dev, tot_dev ? tot_dev : g->d_tot,
                  cnt_dev ? (unsigned long long*)cnt_dev : g->d_cnt, err_dev ? (unsigned long long*)err_dev : g->d_err,
                  nullptr, s);
}

int32_t artes_run_device_flow(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                              double* det_dev, double* tot_dev, uint64_t* cnt_dev, uint64_t* err_dev,
                              double* flow_global_dev, double* flow_latitudinal_dev, void* stream) {
    if (!g || !det_dev) return fail(-22, "null argument");
    HIP_TRY(hipSetDevice(g->device));
    hipStream_t s = (hipStream_t)stream;
    if (!tot_dev) { HIP_TRY(hipMemsetAsync(g->d_tot, 0, 6 * sizeof(double), s)); }
    if (!cnt_dev) { HIP_TRY(hipMemsetAsync(g->d_cnt, 0, ARTES_NUM_COUNTERS * 8, s)); }
    if (!err_dev) { HIP_TRY(hipMemsetAsync(g->d_err, 0, ARTES_NUM_ERR * 8, s)); }
    return launch(g, p, first, n, seed, det_dev, tot_dev ? tot_dev : g->d_tot,
                  cnt_dev ? (unsigned long long*)cnt_dev : g->d_cnt, err_dev ? (unsigned long long*)err_dev : g->d_err,
                  nullptr, s, flow_global_dev, flow_latitudinal_dev);
}


static int32_t run_host(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                        double* det, double* totals, uint64_t* counters, uint64_t* err, double* records,
                        double* flow_global = nullptr, double* flow_latitudinal = nullptr) {
    if (!g || !p) return fail(-22, "null argument");
    HIP_TRY(hipSetDevice(g->device));
    const size_t nc = (size_t)g->T.ncell;
    double *fg = nullptr, *ft = nullptr;
    if (flow_global || flow_latitudinal) {
        if (!g->d_flow) HIP_TRY(hipMalloc((void**)&g->d_flow, 7 * nc * sizeof(double)));
        HIP_TRY(hipMemset(g->d_flow, 0, 7 * nc * sizeof(double)));
        if (flow_global) fg = g->d_flow;
        if (flow_latitudinal) ft = g->d_flow + 3 * nc;
    }
    const size_t stride = (size_t)16 * p->nx * p->ny;
    if (g->out_cap < stride) {
        if (g->d_out) hipFree(g->d_out);
        g->d_out = nullptr;
        HIP_TRY(hipMalloc((void**)&g->d_out, stride * sizeof(double)));
        g->out_cap = stride;
    }
    if (records) {
        const size_t rec_n = std::max<uint64_t>(n, 1) * ARTES_TRACE_FIELDS;
        if (g->rec_cap < rec_n) {
            if (g->d_rec) hipFree(g->d_rec);
            g->d_rec = nullptr;
            HIP_TRY(hipMalloc((void**)&g->d_rec, rec_n * sizeof(double)));
            g->rec_cap = rec_n;
        }
        HIP_TRY(hipMemset(g->d_rec, 0, rec_n * sizeof(double)));
    }
    HIP_TRY(hipMemset(g->d_out, 0, stride * sizeof(double)));
    HIP_TRY(hipMemset(g->d_tot, 0, 6 * sizeof(double)));
    HIP_TRY(hipMemset(g->d_cnt, 0, ARTES_NUM_COUNTERS * 8));
    HIP_TRY(hipMemset(g->d_err, 0, ARTES_NUM_ERR * 8));
    int32_t rc = launch(g, p, first, n, seed, g->d_out, g->d_tot, g->d_cnt, g->d_err, records ? g->d_rec : nullptr, 0, fg, ft);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    if (fg || ft) {
        std::vector<double> hf(7 * nc);
        HIP_TRY(hipMemcpy(hf.data(), g->d_flow, hf.size() * sizeof(double), hipMemcpyDeviceToHost));
        if (flow_global) for (size_t i = 0; i < 3 * nc; i++) flow_global[i] += hf[i];
        if (flow_latitudinal) for (size_t i = 0; i < 4 * nc; i++) flow_latitudinal[i] += hf[3 * nc + i];
    }
    std::vector<double> hd(stride);
    HIP_TRY(hipMemcpy(hd.data(), g->d_out, stride * sizeof(double), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < stride; i++) det[i] += hd[i];
    if (totals) {
        double t2[6];
        HIP_TRY(hipMemcpy(t2, g->d_tot, sizeof(t2), hipMemcpyDeviceToHost));
        const size_t plane = (size_t)p->nx * p->ny;
        for (int k = 0; k < 4; k++) {
            double s = 0.0;
            for (size_t i = 0; i < plane; i++) s += hd[k * plane + i];
            totals[k] += s;
            totals[4 + k] += t2[k];
        }
        totals[8] += t2[4];   // flux_emitted
        totals[9] += t2[5];   // flux_exit
    }
    if (counters) {
        unsigned long long c[ARTES_NUM_COUNTERS];
        HIP_TRY(hipMemcpy(c, g->d_cnt, sizeof(c), hipMemcpyDeviceToHost));
        for (int i = 0; i < ARTES_NUM_COUNTERS; i++) counters[i] += c[i];
    }
    {
        unsigned long long e[ARTES_NUM_ERR];
        HIP_TRY(hipMemcpy(e, g->d_err, sizeof(e), hipMemcpyDeviceToHost));
        if (err)
            for (int i = 0; i < ARTES_NUM_ERR; i++) err[i] += e[i];
        if (e[ARTES_ERR_WATCHDOG]) return fail(-5, "transport kernel watchdog fired: schedule bug, results invalid");
        if (e[ARTES_ERR_LISTS]) return fail(-5, "work-list invariant violated (ARTES_DEBUG check): results invalid");
        if (e[ARTES_ERR_PENDING] || e[ARTES_ERR_CELL])
            return fail(-5, "k_trace trace-state invariant violated (ARTES_DEBUG check: pending bit / cell index): results invalid");
    }
    if (records) HIP_TRY(hipMemcpy(records, g->d_rec, n * ARTES_TRACE_FIELDS * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

int32_t artes_run(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                  double* det, double* totals, uint64_t* counters, uint64_t* err) {
    if (!det) return fail(-22, "null detector");
    return run_host(g, p, first, n, seed, det, totals, counters, err, nullptr);
}

int32_t artes_run_flow(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                       double* det, double* totals, uint64_t* counters, uint64_t* err, double* flow_global,
                       double* flow_latitudinal) {
    if (!det) return fail(-22, "null detector");
    return run_host(g, p, first, n, seed, det, totals, counters, err, nullptr, flow_global, flow_latitudinal);
}

int32_t artes_run_trace(artes_grid* g, const artes_run_params* p, uint64_t first, uint64_t n, uint64_t seed,
                        double* records) {
    if (!g || !p || !records) return fail(-22, "null argument");
    if (n > (1ull << 24)) return fail(-22, "trace runs are limited to 2^24 packets");
    std::vector<double> det((size_t)16 * p->nx * p->ny, 0.0);
    return run_host(g, p, first, n, seed, det.data(), nullptr, nullptr, nullptr, records);
}

const char* artes_last_launch(artes_grid* g) {
    if (!g) return "";
    // (recorded by launch(): "none" for an n = 0 call, or an event-engine call that failed before
    // its first k_trace launch)
    if (g->last_engine == 2) g->launch_info = "persistent";
    else if (g->last_engine == 1 && !g->last_trace.empty()) g->launch_info = g->last_trace + " " + g->last_event;
    else g->launch_info = "none";
    return g->launch_info.c_str();
}

int32_t artes_set_profiling(artes_grid* g, int32_t on) {
    if (!g) return fail(-22, "null grid");
    g->prof = on != 0;
    g->prof_used = 0;
    return 0;
}

int32_t artes_kernel_times(artes_grid* g, double* ms, uint64_t* launches) {
    if (!g || !ms) return fail(-22, "null argument");
    for (int k = 0; k < ARTES_NUM_KERNELS; k++) { ms[k] = 0.0; if (launches) launches[k] = 0; }
    if (g->prof_used == 0) return 0;
    HIP_TRY(hipSetDevice(g->device));
    HIP_TRY(hipEventSynchronize(g->prof_ev[2 * g->prof_used - 1]));
    // (development build: ARTES_LAUNCH_LOG=<file> appends every launch's kind and time, one line per call)
#ifdef ARTES_DEV_KNOBS
    const char* log = getenv("ARTES_LAUNCH_LOG");
    FILE* lf = log ? fopen(log, "a") : nullptr;
#else
    FILE* lf = nullptr;
#endif
    for (size_t i = 0; i < g->prof_used; i++) {
        float t = 0.0f;
        HIP_TRY(hipEventElapsedTime(&t, g->prof_ev[g->prof_start[i]], g->prof_ev[2 * i + 1]));
        ms[g->prof_kind[i]] += (double)t;
        if (launches) launches[g->prof_kind[i]] += 1;
        if (lf) fprintf(lf, "%d:%.4f ", g->prof_kind[i], t);
    }
    if (lf) { fprintf(lf, "\n"); fclose(lf); }
    g->prof_used = 0;
    return 0;
}

double artes_last_kernel_ms(artes_grid* g) {
    if (!g || !g->timed) return -1.0;
    float ms = -1.0f;
    if (hipEventElapsedTime(&ms, g->ev0, g->ev1) != hipSuccess) return -1.0;
    return (double)ms;
}

}  // extern "C"
