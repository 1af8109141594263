// kernel_event.hpp -- the event-based engine ("event", default).
//
// The reference runs one packet per OpenMP thread from emission to exit
// (ARTES.f90:546-955).  On a 64-lane wave that history-based form makes every wave
// execute the union of all lanes' branches, and carrying the whole packet state plus
// the scattering math in one kernel costs ~300 VGPRs (one wave per SIMD).  Here the
// packet life is split at its natural seams into three kernels over a pool of P
// in-flight packets whose state lives in HBM (a 128-byte transport record per packet,
// `Slot`, and a 128-byte diagnostic one, `SlotDiag`):
//
//   k_trace  the hot loop: cell_face steps (ARTES.f90:2800-3470) of every trace --
//            first optical depth (625-656), propagation (689-778, 848-941) and peel-off
//            (4739-4761) -- plus the cheap transitions between them done inline:
//            forced first interaction (660-685) and the scattering-loop head (793-813:
//            roulette, albedo weight, minimum weight).  Lanes refill themselves from the
//            trace list (wave-level grabs on 8 sharded cursors), so lanes stay busy until
//            the list drains.  A segment ends when a peel-off trace ends (-> event list)
//            or the packet ends (-> emit list).
//   k_event  peel-off contribution (4765-4984) + scatter_photon / polarization_rotation
//            (819-846) + the next optical depth; -> trace list.  All lanes run the same
//            branchy math, so nothing is wasted on divergence.
//   k_emit   closes finished packets (per-packet moments, counters, trace records) and
//            emits new packets into the freed slots (emit_photon, 1027-1115) -> trace list.
//
// One host-side iteration = k_trace, k_event, k_emit, k_rotate; iterations repeat until
// the trace list is empty.
#pragma once

#include <cstddef>

#include "device_common.hpp"

namespace artes {

// packet-state pool: two 128-byte records per slot (one cache line each), in two arrays.
// The work lists visit slots in no particular order, so a record layout keeps every
// access of a lane inside its own line; a structure-of-arrays pool would touch one line
// per field per lane.  `Slot` (line 0) holds the whole transport state: every kernel
// reads and writes that line only.  `SlotDiag` (line 1) holds diagnostics -- the
// packet-level moments (R.moments), the trace records (R.rec) -- and the rare
// surface-peel angle, so a production run moves one random line per packet access, and
// the random accesses span the P x 128 B of the transport array only.  Every trace
// starts at the packet position (p*, pcell, pface) with zero accumulated optical depth,
// so no separate trace position is stored.
struct alignas(128) Slot {
    // the transport state, one 128-byte line: every kernel reads and writes only this
    double px, py, pz;                  // packet position (last interaction / emission)
    double dx, dy, dz;                  // packet direction
    double ttgt;                        // target optical depth of a propagation trace
    unsigned long long r0, r1;          // xoroshiro128++ state
    int pcell, pface;                   // packed cell / face of the packet position
    int mode, ncross;
    double wI;                          // Stokes I including the weights applied in k_trace
    double tpeel;                       // optical depth of the last peel-off trace
    double q1, q2, q3;                  // Stokes Q, U, V per unit I as of the last scattering
};
static_assert(sizeof(Slot) == 128, "the transport state is one cache line");

// the rest of a packet's record, in an array of its own so the transport kernels' random
// slot accesses span half the address range (fewer address-translation misses):
// diagnostics and the surface peel
struct alignas(128) SlotDiag {
    double cos_surf;                    // surface peel: cos(normal, detector) (ARTES.f90:4623)
    double cs0, cs1, cs2, cs3;          // moments: running contribution to the current pixel
    double pt0, pt1, pt2, pt3;          // moments: packet total per Stokes
    double peel_sum;                    // trace records: total peeled intensity
    unsigned long long pid;             // trace records: packet id
    int cur_pix, nscat;                 // moments: current pixel; trace records: scatterings
    double peel_pol[3];                 // trace records: peeled -Q, U, V (detector sign, ARTES.f90:4956)
    double spare1;
};
static_assert(sizeof(SlotDiag) == 128, "one line");

// line 0 of a slot as k_event reads it (loaded one event ahead, see k_event)
struct alignas(16) Line0 {
    double px, py, pz, dx, dy, dz, ttgt;
    unsigned long long r0, r1;
    int pcell, pface, mode, ncross;
    double wI, tpeel, q1, q2, q3;
};
static_assert(sizeof(Line0) == 128 && offsetof(Line0, wI) == offsetof(Slot, wI) && offsetof(Line0, q3) == offsetof(Slot, q3),
              "Line0 mirrors line 0 of Slot");

struct Pool {
    int P;
    Slot* __restrict__ s;        // [P] transport state
    SlotDiag* __restrict__ d;    // [P] diagnostics, surface peel
};

// A trace list is read as list index j < split -> position j, j >= split -> position
// P-1-(j-split).  Two orders (R.emit_first):
//  0: k_event's traces at [0, event_n), k_emit's after them (split = the whole list);
//  1: k_emit's traces at the front, k_event's from position P-1 downwards (split =
//     emit_n): the new packets' chains (first optical depth -> propagation -> peel) are
//     handed out first.  Radial-only grids gain 2-6 % from it, ray3d loses 1.5 %.
struct Lists {
    const int* trace_in;  const int* trace_in_n;  const int* trace_in_split;
    int* trace_out;       int* trace_out_n;
    int* event;           int* event_n;
    int* emit;            int* emit_n;
    unsigned int* grab;                 // [8] shard cursors of trace_in
    unsigned long long* next_pkt;       // packets handed out so far
    int* dbg_owner;                     // ARTES_DEBUG: [P] last (iteration, stage) tag per slot
    int* dbg_iter;                      // ARTES_DEBUG: iteration counter (k_rotate)
    int P;                              // trace-list capacity: twice the slots of this sub-engine (L2)
    unsigned long long first, n;        // the packet ids of this sub-engine: [first, first + n)
};

// XCD-partitioned sub-engines.  MI355X dispatches the blocks of a grid round-robin over
// its 8 XCDs, each with its own L2 and address-translation caches.  The pool is split
// into NSUB parts of P / NSUB slots with lists, counters and packet ids of their own, and
// the blocks b of every kernel with b % NSUB == s work on part s only (block b / NSUB of
// the part's b' grid): a slot stays on one XCD for its whole life, and an XCD's random
// record accesses span 1/8 of the pool.  The packet ids [first, first + n) are split into
// NSUB contiguous ranges; results per packet id are unchanged.
constexpr int NSUB = 8;
struct SubLists {
    Lists l[NSUB];
};
// The list counters and shard cursors each on a 256-byte line of their own: device-scope
// atomics are performed at the memory side, and those on one line serialise there -- packed
// [field][NSUB], the trace-out, event and emit counters of all 8 sub-engines and their 64 shard
// cursors shared five lines.
#ifndef ARTES_CNT_PAD
#define ARTES_CNT_PAD 64
#endif
constexpr int CPAD = ARTES_CNT_PAD;   // ints from one counter (cursor) to the next
__host__ __device__ constexpr int grab_at(int sub, int sh) { return (sub * 8 + sh) * CPAD; }
__device__ __forceinline__ int sub_of_block() { return (int)blockIdx.x % NSUB; }
__device__ __forceinline__ int sub_block() { return (int)blockIdx.x / NSUB; }
__device__ __forceinline__ int sub_grid() { return (int)gridDim.x / NSUB; }

// Work-list invariants of one engine iteration (checked by ARTES_DEBUG builds; a
// violation counts error ARTES_ERR_LISTS and fails the run):
//  (L1) every live packet's slot is named exactly once, by one list: the input trace
//       list (k_trace), then the event list or the emit list (k_trace pushes each slot it
//       ends to exactly one), then the output trace list (k_event at its event index,
//       k_emit at event_n + its emit index, or mirrored from position P-1 downwards with
//       emit_first); a slot no list names is free;
//  (L2) list entries are slot ids in [0, S) or -1 (a hole: a dropped or retired packet), S
//       the sub-engine's slots; a trace-list position read is < trace_in_n and maps into
//       [0, P) (the mirrored half: P-1-(j-split), j < trace_in_n); event_n + emit_n <= P,
//       so the two writers of the output trace list never overlap.  The trace lists hold
//       P = 2 S positions: a packet that k_event drops (a peel-off or scattering error)
//       leaves a hole at its event position AND takes an emit position for the slot's next
//       packet, so event_n + emit_n reaches 2 S when every event drops -- with S positions
//       the emit half ran past the list (round 3: the oblate star source, where the
//       reference's emission fails for every packet, faulted with a call-sized pool);
//  (L3) a slot's mode matches its list: a trace kind in the trace list, S_PEEL_DONE /
//       S_SURF_HIT in the event list, an end state (or S_FRESH at the start) in the emit list.
// A variant that parks unfinished traces of k_trace's tail must give them list positions
// of their own (outside [0, event_n + emit_n)) and persist the trace state it drops; both
// appending them with an atomic counter into positions the other writers also use, and
// resuming them with the in-register trace state lost, break (L1)/(L2) -- duplicate slots
// (the trajectory mismatch) and mirrored positions outside [0, P) (a memory fault).
__device__ __forceinline__ void dbg_claim(const DevRun& R, const Lists& L, int slot, int P, int stage, bool mode_ok) {
#ifdef ARTES_DEBUG
    if (slot < -1 || slot >= P || (slot >= 0 && !mode_ok)) { atomicAdd(&R.err[ARTES_ERR_LISTS], 1ULL); return; }
    if (slot >= 0) {
        const int tag = 3 * *L.dbg_iter + stage;
        if (atomicExch(&L.dbg_owner[slot], tag) == tag) atomicAdd(&R.err[ARTES_ERR_LISTS], 1ULL);
    }
#endif
}

// slot modes
enum SlotMode : int {
    S_FRESH = 0,        // never held a packet
    S_FIRST = 1, S_PROP = 2, S_PEEL = 3,       // trace kinds (in a trace list)
    S_PEEL_DONE = 4,    // in the event list; bit 8 = exit, bit 9 = cell error, bits 10-11 = peel kind
    S_END_EXIT = 5, S_END_ABS = 6, S_END_DROP = 7,   // in the emit list
    S_RETIRED = 8,
    S_PEEL_T = 9,       // trace: thermal emission peel-off (peel_thermal, ARTES.f90:4519-4598)
    S_PEEL_S = 10,      // trace: surface peel-off (peel_surface, ARTES.f90:4600-4708)
    S_SURF_HIT = 11,    // in the event list: Lambertian reflection pending (ARTES.f90:764-772)
};
constexpr int FLAG_EXIT = 1 << 8;
constexpr int FLAG_ERR = 1 << 9;
constexpr int PEEL_KIND_SHIFT = 10;   // 0 = after scattering, 1 = thermal, 2 = surface

__device__ __forceinline__ bool is_peel_trace(int mode) { return mode == S_PEEL || mode == S_PEEL_T || mode == S_PEEL_S; }
// Emit-list entries carry the ended packet's state in bits 27-28 (0: a fresh slot, its
// record says what it is; 1-3: S_END_EXIT / S_END_ABS / S_END_DROP), so k_emit counts
// the ends without a dependent read of the record (slots < 2^26, checked at pool size).
__device__ __forceinline__ int emit_entry(int slot, int mode) {
    return slot | ((mode >= S_END_EXIT && mode <= S_END_DROP ? mode - S_END_EXIT + 1 : 0) << 27);
}

__device__ __forceinline__ bool to_event_list(int end) {
    const int b = end & 0xFF;
    return b == S_PEEL_DONE || b == S_SURF_HIT;
}

__device__ __forceinline__ int pack_cell(int r, int t, int p) { return r | (t << 12) | (p << 22); }
__device__ __forceinline__ void unpack_cell(int c, int& r, int& t, int& p) { r = c & 0xFFF; t = (c >> 12) & 0x3FF; p = (c >> 22) & 0x3FF; }
__device__ __forceinline__ int pack_face(int type, int idx) { return (type << 28) | (idx & 0x0FFFFFFF); }
__device__ __forceinline__ void unpack_face(int f, int& type, int& idx) { type = (f >> 28) & 0xF; idx = f & 0x0FFFFFFF; if (idx == 0x0FFFFFFF) idx = -1; }

// Work distribution over the trace list: the first `n_static` entries are split into
// 64-entry chunks dealt round-robin to the waves (chunk w, w+W, w+2W, ... for wave w; no
// atomics, a wave-local cursor), the rest is grabbed dynamically through 8 sharded
// cursors to balance the tail.  Device-scope atomics are resolved at the memory side
// (~µs round trip), so a purely dynamic grab stalls every refill.  The list arrives in
// the order packets finished their previous trace, which correlates with how long their
// next trace runs; dealing chunks round-robin gives every wave a sample of the whole list.
struct TraceCursor {
    int pos, end;              // current static chunk of this wave (wave-uniform)
    int chunk, nchunk, stride; // chunk index, static chunk count, waves in the grid
    int dyn_lo, dyn_n;         // dynamic range
    int pf;                    // list entries [.., pf) of the current chunk have their records prefetched
    int dpos, dend;            // the rest of this wave's last dynamic grab (list indices)
    int dead;                  // bit s: dynamic shard s is used up (no more atomics on it)
    bool exhausted;
};

// list index j -> list position (see Lists: j < split from the front, the rest mirrored)
__device__ __forceinline__ int list_pos(int j, int split, int P) { return j < split ? j : P - 1 - (j - split); }

// Lookahead of the static deal (k_trace).  A refill used to wait for two dependent memory
// round trips: the list entry (the slot id), then the slot's record, a random line of the
// pool (HBM and an address-translation miss).  Now every lane holds the slot id of one entry
// of the wave's current static chunk (`ck_cur`, lane i: list index chunk * 64 + i) and of the
// next one (`ck_nxt`, loaded a whole chunk ahead), so a static take reads its slot ids from
// its own wave (ds_bpermute); and after each take the records of the chunk's next entries --
// the next refill's -- are prefetched into L2 (`prefetch_line`), so that refill's record loads
// hit L2 about ten iterations later.  The dynamic part still loads list entries directly.
__device__ __forceinline__ int load_chunk(const int* list, int chunk, int nchunk, int split, int P) {
    return chunk < nchunk ? list[list_pos(chunk * 64 + (int)(threadIdx.x & 63), split, P)] : -1;
}
// A load whose data nobody reads: the line (and its address translation) moves into L2.  It
// is an LDS-DMA load (no VGPR destination, so no register can be reused under the returning
// data) into a 256-byte LDS scratch area that nothing reads (`lds_sink`, the LDS byte address);
// the compiler does not see it, so it places no wait for it (its own vmcnt waits only get
// stricter: memory operations complete in issue order).  M0 is set and restored inside the
// statement (the compiler owns it).  prefetch_drain: before the kernel ends, so no DMA write
// lands in LDS the next block may own.
__device__ __forceinline__ void prefetch_line(const void* p, unsigned lds_sink) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(p), "s"(lds_sink));
}
__device__ __forceinline__ void prefetch_drain() { asm volatile("s_waitcnt vmcnt(0)"); }

__device__ __forceinline__ TraceCursor make_cursor(int n, int static_q64) {
    const int W = sub_grid() * (BLOCK / 64);            // the waves of this sub-engine
    // (the wave index through readfirstlane: the compiler then knows the cursor is
    // wave-uniform, so k_trace's loop, which ends on it, is a uniform loop -- no exec-mask
    // bookkeeping at its latch)
    const int w = __builtin_amdgcn_readfirstlane(sub_block() * (BLOCK / 64) + (int)(threadIdx.x >> 6));
    const int nchunk = (int)((((long long)n * static_q64) >> 6) >> 6);
    TraceCursor c;
    c.chunk = w;
    c.nchunk = nchunk;
    c.stride = W;
    c.pos = w * 64;
    c.end = (w < nchunk) ? c.pos + 64 : c.pos;
    c.dyn_lo = nchunk * 64;
    c.dyn_n = n - nchunk * 64;
    c.pf = c.pos;
    c.dpos = 0;
    c.dend = 0;
    c.dead = 0;
    c.exhausted = (n == 0);
    return c;
}

// hand out up to popc(need) list indices to the lanes with `need`; returns this lane's or -1
// a wave's cursor kept in LDS, read back as wave-uniform (scalar) values
__device__ __forceinline__ TraceCursor load_cursor(const TraceCursor* p) {
    TraceCursor c;
    c.pos = __builtin_amdgcn_readfirstlane(p->pos);
    c.end = __builtin_amdgcn_readfirstlane(p->end);
    c.chunk = __builtin_amdgcn_readfirstlane(p->chunk);
    c.nchunk = __builtin_amdgcn_readfirstlane(p->nchunk);
    c.stride = __builtin_amdgcn_readfirstlane(p->stride);
    c.dyn_lo = __builtin_amdgcn_readfirstlane(p->dyn_lo);
    c.dyn_n = __builtin_amdgcn_readfirstlane(p->dyn_n);
    c.pf = __builtin_amdgcn_readfirstlane(p->pf);
    c.dpos = __builtin_amdgcn_readfirstlane(p->dpos);
    c.dend = __builtin_amdgcn_readfirstlane(p->dend);
    c.dead = __builtin_amdgcn_readfirstlane(p->dead);
    c.exhausted = __builtin_amdgcn_readfirstlane((int)p->exhausted) != 0;
    return c;
}

// Hands out up to popc(need) list indices to the lanes with `need`; returns this lane's or -1.
// LA (k_trace's lookahead, above): a static entry's slot id comes from the chunk registers
// (`slot`; -2: load it from the list), and the records of the chunk's next PF entries are
// prefetched.  Call with the whole wave active.
// Dynamic part: an atomic grab asks for at least `grab` entries and the wave keeps what its
// lanes do not need now (dpos, dend) for its next refills, and a shard found used up is not
// asked again (`dead`).  A device-scope atomic is a memory-side round trip of a few
// microseconds, and the grab used to ask for exactly the lanes' need, one to eight shards in a
// row: a k_trace wave spent 5 % (bench grid) to 9 % (cloudy) of its time in the take.
template <bool LA = false>
__device__ __forceinline__ int wave_take(TraceCursor& c, unsigned int* cursors, int home, bool need, int grab, int* slot = nullptr,
                                         int* ck_cur = nullptr, int* ck_nxt = nullptr, const Lists* L = nullptr, int split = 0,
                                         const Slot* rec = nullptr, unsigned lds_sink = 0, int* n_atom = nullptr) {
    constexpr int PF = 32;
    const int lane = threadIdx.x & 63;
    const unsigned long long mask = __ballot(need);
    const int k = __popcll(mask);
    const int rank = __popcll(mask & ((1ULL << lane) - 1ULL));
    int got = 0, mine = -1;
    if constexpr (LA) *slot = -2;
    if (c.pos < c.end) {
        for (int part = 0; part < 2 && got < k && c.pos < c.end; part++) {   // current chunk, then the next
            const int take = min(k - got, c.end - c.pos);
            if constexpr (LA) {
                const int s = __shfl(*ck_cur, (c.pos - c.chunk * 64 + rank - got) & 63);
                if (need && rank >= got && rank < got + take) *slot = s;
            }
            if (need && rank >= got && rank < got + take) mine = c.pos + (rank - got);
            got += take;
            c.pos += take;
            if (c.pos == c.end) {
                c.chunk += c.stride;
                c.pos = c.chunk * 64;
                c.end = (c.chunk < c.nchunk) ? c.pos + 64 : c.pos;
                c.pf = c.pos;
                if constexpr (LA) {
                    *ck_cur = *ck_nxt;
                    *ck_nxt = load_chunk(L->trace_in, c.chunk + c.stride, c.nchunk, split, L->P);
                }
            }
        }
        if constexpr (LA) {
            // the next refill's records: entries [max(pos, pf), pos + PF) of the current chunk
            const int lo = max(c.pos, c.pf), hi = min(c.end, c.pos + PF);
            if (lo < hi) {
                const int s = __shfl(*ck_cur, (lo - c.chunk * 64 + lane) & 63);
                if (lane < hi - lo && s >= 0) prefetch_line(rec + s, lds_sink);
                c.pf = hi;
            }
        }
        return mine;
    }
    if (c.dpos < c.dend) {   // the rest of the last grab
        const int take = min(k, c.dend - c.dpos);
        if (need && rank < take) mine = c.dpos + rank;
        got = take;
        c.dpos += take;
    }
    for (int a = 0; a < 8 && got < k; a++) {
        const int sh = (home + a) & 7;
        if ((c.dead >> sh) & 1) continue;
        const int lo = c.dyn_lo + (int)(((long long)c.dyn_n * sh) >> 3);
        const int hi = c.dyn_lo + (int)(((long long)c.dyn_n * (sh + 1)) >> 3);
        if (hi <= lo) {
            c.dead |= 1 << sh;
            continue;
        }
        const int want = k - got;
        const int req = max(want, grab);
        unsigned int base = 0;
        if (lane == 0) base = atomicAdd(&cursors[sh * CPAD], (unsigned int)req);
        if (n_atom) ++*n_atom;   // (timing build: the grabs a take issued)
        base = __builtin_amdgcn_readlane(base, 0);   // (uniform: an SGPR)
        const long long start = (long long)lo + base;
        const int all = (int)max(0LL, min((long long)req, (long long)hi - start));
        const int avail = min(want, all);
        if (need && rank >= got && rank < got + avail) mine = (int)start + (rank - got);
        got += avail;
        if (all > avail) {   // (got == k now: the loop ends)
            c.dpos = (int)start + avail;
            c.dend = (int)start + all;
        }
        if (all < req) c.dead |= 1 << sh;
    }
    if (got == 0 && k > 0) c.exhausted = true;
    return mine;
}

// Wave-aggregated append of this lane's `val` (if `want`) to a global list: one atomic
// per wave instead of one per lane.  Same-address device-scope atomics are serialised
// at the memory side (the L2s of the 8 XCDs are not coherent), so per-lane appends to
// the list counters would cost ~10 ns per packet event.
__device__ __forceinline__ void wave_append(bool want, int val, int* list, int* list_n) {
    const unsigned long long mask = __ballot(want);
    if (mask == 0) return;
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (lane == __ffsll((long long)mask) - 1) base = atomicAdd(list_n, __popcll(mask));
    base = __shfl(base, __ffsll((long long)mask) - 1);
    if (want) list[base + __popcll(mask & ((1ULL << lane) - 1ULL))] = val;
}

// Per-wave LDS staging queue in front of a global list, for producers whose lanes finish at
// scattered times (k_trace): QCAP entries, flushed with one atomic once QFLUSH or more wait
// (`flush_if`, called where the atomic's round trip is off the critical path: with
// QFLUSH + 64 <= QCAP a push of up to 64 entries never has to flush first).  Every wave of a
// sub-engine flushes into the same counter, and same-address atomics serialise at the
// memory side: flushing every 192 entries instead of every 64 took iso's k_trace from 196.6
// to 162.5 ms per 3e8 packets (hg -0.5 %, cloudy -1 %, ray3d the same); 512 and 1024
// measured the same as 256 (profiles/r03/queue_size_ab.txt).
#ifndef ARTES_QCAP
#define ARTES_QCAP 256
#endif
#ifndef ARTES_QFLUSH
#define ARTES_QFLUSH 192
#endif
constexpr int QCAP = ARTES_QCAP, QFLUSH = ARTES_QFLUSH;
static_assert(QFLUSH + 64 <= QCAP, "a push of 64 entries fits without a flush");
struct WaveQueue {
    int* buf;     // this wave's QCAP LDS entries
    int cnt;      // wave-uniform fill level
    __device__ __forceinline__ void flush(int* list, int* list_n) {
        if (cnt == 0) return;
        const int lane = threadIdx.x & 63;
        int base = 0;
        if (lane == 0) base = atomicAdd(list_n, cnt);
        base = __shfl(base, 0);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < QCAP / 64; k++)   // (unrolled: a counted loop here cost k_trace 18 registers and spills)
            if (lane + 64 * k < cnt) list[base + lane + 64 * k] = buf[lane + 64 * k];
        __builtin_amdgcn_wave_barrier();
        cnt = 0;
    }
    __device__ __forceinline__ void flush_if(int at, int* list, int* list_n) {
        if (cnt >= at) flush(list, list_n);
    }
    __device__ __forceinline__ void push(bool want, int val) {
        const unsigned long long mask = __ballot(want);
        const int k = __popcll(mask);
        if (k == 0) return;
        const int lane = threadIdx.x & 63;
        if (want) buf[cnt + __popcll(mask & ((1ULL << lane) - 1ULL))] = val;
        __builtin_amdgcn_wave_barrier();
        cnt += k;
    }
};

// park the packet in a new propagation trace starting at its position (an interaction
// point: no face; the field carried the matrix id, see event_one)
__device__ __forceinline__ void start_prop(const Pool& S, int slot, double tau) {
    S.s[slot].ttgt = tau;
    S.s[slot].pface = 0;
    S.s[slot].mode = S_PROP;
}

// detector pixel of a peel from (px, py, pz) (ARTES.f90:4947-4951); -1 outside the image
__device__ __forceinline__ int peel_pixel(const DevRun& R, double px, double py, double pz) {
    const double x_im = py * R.cdp - px * R.sdp;
    const double y_im = pz * R.sdt - py * R.cdt * R.sdp - px * R.cdt * R.cdp;
    const int ix = (int)((double)R.nx * (x_im + R.x_max) / (2.0 * R.x_max));
    const int iy = (int)((double)R.ny * (y_im + R.y_max) / (2.0 * R.y_max));
    if (ix < 0 || ix >= R.nx || iy < 0 || iy >= R.ny) return -1;
    return iy * R.nx + ix;
}

// Detector accumulation of k_event: planes 0-8 (I Q U V sums, their squares, the peel
// count) go to `acc` (the block's LDS detector or its HBM copy), plane 9 (the I-only peel
// count) and the packet moments 12-15 to `det` (the block's HBM copy).  With a one-pixel
// detector (spectrum / phase, ARTES.f90:453-465) every peel of the grid would add to the
// same ten addresses, so PIX1 keeps per-lane partial sums instead -- in the lane's own
// LDS slot (ten doubles, stride = the block size: conflict-free; registers would take the
// kernel past 168 VGPRs, i.e. 2 waves per SIMD) -- and reduces them over the wave once, at
// the end of the kernel (ARTES.f90:4953-4972 sums).
// Reproducible accumulation (tuning "det_ordered", DM_ORD): the floating-point sums above depend
// on the order in which the dynamically scheduled events reach each address, so two identical
// runs differ in the last bits.  Integer addition is associative: each contribution is rounded
// once to a 128-bit fixed-point integer, round(|v| 2^80) with v's sign (resolution 2^-80 ~ 8e-25,
// range 2^47; contributions are packet weights of order 1), and added with two 64-bit integer
// atomics -- the low word with the old value returned, its carry into the high word -- so every
// schedule ends with the same bits.  reduce_fixed sums the copies in integers and converts once.
__device__ __forceinline__ void fix_add(unsigned long long* e, double v) {
    const double a = fmin(fabs(v), 0x1p46) * 0x1p80;      // (exact scaling; |v| beyond 2^46 saturates)
    const double hd = floor(a * 0x1p-64);
    const double r = a - hd * 0x1p64;                      // (exact: a's bits below 2^64)
    unsigned long long lo = (unsigned long long)rint(r), hi = (unsigned long long)(long long)hd;
    if (v < 0.0) {   // two's complement of the 128-bit value
        hi = ~hi + (lo == 0 ? 1ull : 0ull);
        lo = 0ull - lo;
    }
    if ((lo | hi) == 0) return;
    const unsigned long long old = atomicAdd(e, lo);
    atomicAdd(e + 1, hi + (old + lo < old ? 1ull : 0ull));
}

// Detector accumulation of k_event: planes 0-8 (I Q U V sums, their squares, the peel
// count) go to `acc` (the block's LDS detector or its HBM copy), plane 9 (the I-only peel
// count) and the packet moments 12-15 to `det` (the block's HBM copy).  With a one-pixel
// detector (spectrum / phase, ARTES.f90:453-465) every peel of the grid would add to the
// same ten addresses, so PIX1 keeps per-lane partial sums instead -- in the lane's own
// LDS slot (ten doubles, stride = the block size: conflict-free; registers would take the
// kernel past 168 VGPRs, i.e. 2 waves per SIMD) -- and reduces them over the wave once, at
// the end of the kernel (ARTES.f90:4953-4972 sums).  DM_ORD: planes 0-9 as fixed-point
// integers in the block's copy of R.fix (fix_add).
enum : int { DM_ATOM = 0, DM_PIX1 = 1, DM_ORD = 2 };
template <int DM>
struct DetAcc {
    double* __restrict__ det;
    double* __restrict__ acc;
    size_t plane;
    double* __restrict__ lane;   // PIX1: this lane's slot, lane[k * stride] (planes 0-7)
    int stride;
    uint32_t n8;                 // PIX1: the lane's peel count (plane 8 adds 1 per peel): a register
    unsigned long long* __restrict__ fix;   // DM_ORD: the block's fixed-point copy
    __device__ __forceinline__ void init(double* d, double* a, size_t pl, double* slots = nullptr, int nthreads = 0,
                                         unsigned long long* f = nullptr) {
        det = d; acc = a; plane = pl; fix = f;
        n8 = 0;
        if constexpr (DM == DM_PIX1) {
            lane = slots + threadIdx.x; stride = nthreads;
#pragma unroll
            for (int k = 0; k < 8; k++) lane[k * stride] = 0.0;
        }
    }
    // (plane 8 takes v = 1 at its call site: a peel's count; plane 9 -- the I-only count of the
    // rare thermal / surface peels -- goes to the HBM copy at once)
    __device__ __forceinline__ void add(int k, int pix, double v) {
        if constexpr (DM == DM_PIX1) {
            if (k == 8) n8++;
            else if (k == 9) unsafeAtomicAdd(&det[9 * plane], v);
            else lane[k * stride] += v;
        }
        else if constexpr (DM == DM_ORD) fix_add(fix + 2 * ((size_t)k * plane + pix), v);
        else if (k == 9) unsafeAtomicAdd(&det[9 * plane + pix], v);   // rare (thermal / surface)
        else unsafeAtomicAdd(&acc[k * plane + pix], v);
    }
    // PIX1: one wave-reduced add per plane (call with the whole wave)
    __device__ __forceinline__ void flush_wave() {
        if constexpr (DM == DM_PIX1) {
#pragma unroll
            for (int k = 0; k < 9; k++) {
                const double v = k < 8 ? wave_sum_f64(lane[k * stride]) : (double)wave_sum_u64(n8);
                if ((threadIdx.x & 63) == 0 && v != 0.0) unsafeAtomicAdd(&det[k * plane], v);
            }
        }
    }
};

// LDS bytes of the PIX1 per-lane slots of a k_event block (planes 0-7; the counts are registers)
__host__ __device__ inline size_t pix1_slot_bytes(int block) { return (size_t)8 * block * sizeof(double); }

// a peel that carries Stokes I only (peel_thermal 4577-4583, peel_surface 4684-4690):
// moments 0 and 4, and the I-only count plane 9 (the reference counts it for I alone)
template <int DM>
__device__ __forceinline__ void add_peel_I(const DevRun& R, const Pool& S, int slot, DetAcc<DM>& D, double v, int err_code,
                                           uint32_t& c_det) {
    if (!(v > 0.0 && v < 1.e100)) { log_err(R, err_code); return; }
    const int pix = peel_pixel(R, S.s[slot].px, S.s[slot].py, S.s[slot].pz);
    if (pix < 0) { log_err(R, 63); return; }
    D.add(0, pix, v);
    D.add(4, pix, v * v);
    D.add(9, pix, 1.0);
    double* __restrict__ det = D.det;
    const size_t plane = D.plane;
    if (R.moments) {
        const int cur = S.d[slot].cur_pix;
        double cs[4] = {S.d[slot].cs0, S.d[slot].cs1, S.d[slot].cs2, S.d[slot].cs3};
        if (pix != cur) {
            if (cur >= 0) {
#pragma unroll
                for (int q = 0; q < 4; q++) unsafeAtomicAdd(&det[(12 + q) * plane + cur], cs[q] * cs[q]);
            }
            S.d[slot].cur_pix = pix;
            cs[0] = cs[1] = cs[2] = cs[3] = 0.0;
        }
        S.d[slot].cs0 = cs[0] + v; S.d[slot].cs1 = cs[1]; S.d[slot].cs2 = cs[2]; S.d[slot].cs3 = cs[3];
        S.d[slot].pt0 += v;
    }
    if (R.rec) S.d[slot].peel_sum += v;
    c_det++;
}

// outward unit normal of the (oblate) surface at (x, y, z) (ARTES.f90:1378-1384)
__device__ __forceinline__ void surface_normal(const DevGrid& G, double x, double y, double z, double& n0, double& n1, double& n2) {
    n0 = x / (G.ox * G.ox); n1 = y / (G.oy * G.oy); n2 = z / (G.oz * G.oz);
    const double norm = dsqrt(n0 * n0 + n1 * n1 + n2 * n2);
    n0 /= norm; n1 /= norm; n2 /= norm;
}

// thermal-emission peel done (ARTES.f90:599-622, 4566-4591), then the first optical
// depth trace of the packet; returns 1 (next trace) or 2 (dropped)
template <int DM>
__device__ __forceinline__ int event_thermal(const DevRun& R, const Pool& S, int slot, DetAcc<DM>& D, uint32_t& c_det) {
    const int m = S.s[slot].mode;
    if (m & FLAG_ERR) { log_err(R, 47); S.s[slot].mode = S_END_DROP; return 2; }
    const double tau = S.s[slot].tpeel;
    if ((m & FLAG_EXIT) && tau < 50.0)
        add_peel_I(R, S, slot, D, exp(-tau) / (4.0 * PI) * S.s[slot].wI, 51, c_det);
    S.s[slot].mode = S_FIRST;
    return 1;
}

// Lambertian reflection (ARTES.f90:1369-1402) at the surface point stored in the slot by
// k_trace, then the surface peel trace if the detector sees the surface element
// (4616-4631), else straight back to the interrupted propagation trace
__device__ __forceinline__ int event_surface_hit(const DevGrid& G, const DevRun& R, const Pool& S, int slot) {
    const double px = S.s[slot].px, py = S.s[slot].py, pz = S.s[slot].pz;
    double n0, n1, n2;
    surface_normal(G, px, py, pz, n0, n1, n2);
    Rng rng; rng.s0 = S.s[slot].r0; rng.s1 = S.s[slot].r1;
    const double alpha = dsqrt(rng.uni());
    const double beta = TWO_PI * rng.uni();
    double e0, e1, e2;
    direction_cosine(R, alpha, beta, n0, n1, n2, e0, e1, e2);
    S.s[slot].r0 = rng.s0; S.s[slot].r1 = rng.s1;
    S.s[slot].dx = e0; S.s[slot].dy = e1; S.s[slot].dz = e2;
    // the surface depolarises (ARTES.f90:1396-1400); I (wI) carries k_trace's weights
    S.s[slot].q1 = 0.0; S.s[slot].q2 = 0.0; S.s[slot].q3 = 0.0;
    // cos of the angle between the surface normal and the detector (4623-4625)
    const double cos_angle = n0 * R.det0 + n1 * R.det1 + n2 * R.det2;
    S.d[slot].cos_surf = cos_angle;
    S.s[slot].mode = cos_angle > 0.0 ? S_PEEL_S : S_PROP;
    return 1;
}

// surface peel done (ARTES.f90:4633-4700), then the interrupted propagation resumes
template <int DM>
__device__ __forceinline__ int event_surface_peel(const DevRun& R, const Pool& S, int slot, DetAcc<DM>& D, uint32_t& c_det) {
    const int m = S.s[slot].mode;
    const double tau = S.s[slot].tpeel;
    if (!(m & FLAG_ERR) && (m & FLAG_EXIT) && tau < 50.0)
        add_peel_I(R, S, slot, D, exp(-tau) * S.d[slot].cos_surf / PI * S.s[slot].wI, 52, c_det);
    S.s[slot].mode = S_PROP;
    return 1;
}

// Layout of the scattering tables a k_event reads: global memory [180][16] matrices and
// [181][4] cumulative tables, or the LDS copies padded to odd row strides of 17 and 5
// doubles.  A matrix row is 128 B, so with stride 16 element e of every row falls in the
// same pair of LDS banks ((a/4) mod 64 for 8-byte reads): lanes interpolating different
// angles -- the usual case -- serialised up to 16-way on every element read (measured:
// LDS bank-conflict cycles ~45 % of k_event's).  Stride 17 (34 dwords) spreads rows over
// 32 bank pairs; stride 5 does the same for the cumulative-table probes.
template <bool PAD>
struct TabLayout {
    static constexpr int RS = PAD ? 17 : 16;            // matrix row stride
    static constexpr int MAT = NANG * RS;               // doubles per matrix
    static constexpr int RS4 = PAD ? 5 : 4;             // row stride of the symmetric form (DevGrid::msym)
    static constexpr int MAT4 = NANG * RS4;
    static constexpr int CS = PAD ? 5 : 4;              // cumulative-table entry stride
    static constexpr int CUM = PAD ? cum_lds_doubles() : (NANG + 1) * CS;   // doubles per cumulative table (cum_at)
};

// Development timing build (-DARTES_DEBUG_TIMING): shader-clock cycles of k_event's regions,
// summed per wave (its first active lane) into `ev_tm` (LDS) and added to error slots 20-27 at
// the end of the kernel (the run's error codes are void): 20 the latch copy (the wait for the
// prefetched record), 21 the whole event, 22 the peel, 23 the angle sampling, 24 the rest of the
// scattering (direction, matrix, rotation, record writes), 25 list writes after the event,
// 26 events, 27 the loop total (tools/time_regions.py)
#ifdef ARTES_DEBUG_TIMING
__device__ __forceinline__ unsigned long long ev_tick() {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t = __builtin_readcyclecounter();
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
__device__ __forceinline__ void ev_add(unsigned long long* tm, int k, unsigned long long d) {
    if ((int)(threadIdx.x & 63) == __builtin_ctzll(__ballot(true))) tm[k] += d;
}
#define EV_TICK(v) const unsigned long long v = ev_tick()
#define EV_ADD(k, d) ev_add(ev_tm, k, d)
#else
#define EV_TICK(v)
#define EV_ADD(k, d)
#endif

// one peel-off + scattering event; returns 1 (next trace) or 2 (packet ended); the peel
// contribution goes to `D` (see DetAcc)
template <int DM, bool PAD, bool PADC = PAD>
__device__ __forceinline__ int event_one(const DevGrid& G, const DevRun& R, const Pool& S, int slot, const Line0& L0,
                                         DetAcc<DM>& D, uint32_t& c_scat, uint32_t& c_det
#ifdef ARTES_DEBUG_TIMING
                                         , unsigned long long* ev_tm
#endif
                                         ) {
    {
        double* __restrict__ det = D.det;
        const size_t plane = D.plane;
        const int m = L0.mode;
        if ((m & 0xFF) == S_SURF_HIT) return event_surface_hit(G, R, S, slot);
        const int kind = (m >> PEEL_KIND_SHIFT) & 3;
        if (kind == 1) return event_thermal(R, S, slot, D, c_det);
        if (kind == 2) return event_surface_peel(R, S, slot, D, c_det);
        if (m & FLAG_ERR) { S.s[slot].mode = S_END_DROP; return 2; }
        const double px = L0.px, py = L0.py, pz = L0.pz;
        double dx = L0.dx, dy = L0.dy, dz = L0.dz;
        // k_trace scaled I by the forced-first-interaction and albedo weights (ARTES.f90:
        // 674-676, 801-807); the polarised components follow by the same factor
        const double wI = L0.wI;
        double st[4] = {wI, L0.q1 * wI, L0.q2 * wI, L0.q3 * wI};
        // the interaction cell's matrix id, left in the face field by k_trace's interaction
        // block (an interaction point lies on no face; reset below when the next trace starts)
        const int mid = G.nmat == 1 ? 0 : L0.pface;
        using TL = TabLayout<PAD>;     // the matrices
        using TC = TabLayout<PADC>;    // the cumulative sampling tables
        const bool sym = G.msym != 0;
        const double* __restrict__ P = G.mats + (size_t)mid * (sym ? TL::MAT4 : TL::MAT);
        const double tau_peel = L0.tpeel;
        // the incoming direction's azimuth, as its cosine and sine (azimuth_cs): the peel-off's
        // phi_old (ARTES.f90:4868-4870) and the scattering's (direction_cosine, 1975-1977)
        double cpo, spo;
        azimuth_cs(dx, dy, cpo, spo);
        bool drop = false;
        EV_TICK(tp0);
        if ((m & FLAG_EXIT) && tau_peel < 50.0) {
            const double w = exp(-tau_peel);
            double mu = dx * R.det0 + dy * R.det1 + dz * R.det2;
            if (mu >= 1.0) mu = 1.0 - 1.e-10;
            else if (mu <= -1.0) mu = -1.0 + 1.e-10;
            double sc[16];
            interp_matrix<TL::RS, TL::RS4>(P, sym, acos(mu), sc);
            double so[4] = {0, 0, 0, 0};
            const bool have_out = peel_rotation(R, dz, mu, cpo, spo, st, sc, so, drop);
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
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            D.add(q, pix, v[q]);
                            D.add(4 + q, pix, v[q] * v[q]);
                        }
                        D.add(8, pix, 1.0);
                        if (R.moments) {   // packet-level moments (diagnostics, line 1)
                            const int cur = S.d[slot].cur_pix;
                            double cs[4] = {S.d[slot].cs0, S.d[slot].cs1, S.d[slot].cs2, S.d[slot].cs3};
                            if (pix != cur) {
                                if (cur >= 0) {
#pragma unroll
                                    for (int q = 0; q < 4; q++) unsafeAtomicAdd(&det[(12 + q) * plane + cur], cs[q] * cs[q]);
                                }
                                S.d[slot].cur_pix = pix;
                                cs[0] = cs[1] = cs[2] = cs[3] = 0.0;
                            }
                            S.d[slot].cs0 = cs[0] + v[0]; S.d[slot].cs1 = cs[1] + v[1];
                            S.d[slot].cs2 = cs[2] + v[2]; S.d[slot].cs3 = cs[3] + v[3];
                            S.d[slot].pt0 += v[0]; S.d[slot].pt1 += v[1]; S.d[slot].pt2 += v[2]; S.d[slot].pt3 += v[3];
                        }
                        if (R.rec) {
                            S.d[slot].peel_sum += wI;
                            S.d[slot].peel_pol[0] += v[1]; S.d[slot].peel_pol[1] += v[2]; S.d[slot].peel_pol[2] += v[3];
                        }
                        c_det++;
                    }
                } else {
                    log_err(R, 53);
                }
            }
        }
        EV_TICK(tp1);
        EV_ADD(22, tp1 - tp0);
        if (drop) { S.s[slot].mode = S_END_DROP; return 2; }
        // scatter_photon + polarization_rotation (ARTES.f90:819-846)
        c_scat++;
        if (R.rec) S.d[slot].nscat += 1;
        Rng rng; rng.s0 = L0.r0; rng.s1 = L0.r1;
        double alpha, beta, c2b, s2b, adeg;
        sample_angles<TC::CS>(G, R, G.cums + (size_t)mid * TC::CUM, rng, st, alpha, beta, c2b, s2b, &adeg);
#ifdef ARTES_DEBUG_TIMING
        asm volatile("" ::"v"(alpha), "v"(beta));   // (the sampling's result: its waits inside the region)
#endif
        EV_TICK(tp2);
        EV_ADD(23, tp2 - tp1);
        double e0, e1, e2;
        direction_cosine_cs(R, alpha, beta, dx, dy, dz, cpo, spo, e0, e1, e2);
        // the matrix at the sampled angle itself (degrees), not at acos(cos(angle)) (ARTES.f90:
        // 1448-1450): the same bin and fraction to ~1e-14
        double sc[16];
        interp_matrix_deg<TL::RS, TL::RS4>(P, sym, adeg, sc);
        if (fabs(alpha) < 1.0) {
            double sn[4];
            polarization_rotation<true>(R, alpha, beta, st, sc, dz, e2, sn, false, c2b, s2b);
            const double inv = sn[0] != 0.0 ? 1.0 / sn[0] : 0.0;
            S.s[slot].q1 = sn[1] * inv; S.s[slot].q2 = sn[2] * inv; S.s[slot].q3 = sn[3] * inv;
            S.s[slot].wI = sn[0];
            S.s[slot].dx = e0; S.s[slot].dy = e1; S.s[slot].dz = e2;
            const double xi = rng.uni();
            S.s[slot].r0 = rng.s0; S.s[slot].r1 = rng.s1;
            start_prop(S, slot, -log(1.0 - xi));
            EV_TICK(tp3);
            EV_ADD(24, tp3 - tp2);
            return 1;
        } else {
            log_err(R, 50);
            S.s[slot].r0 = rng.s0; S.s[slot].r1 = rng.s1;
            S.s[slot].mode = S_END_DROP;
            return 2;
        }
    }
}

// doubles of LDS holding the scattering tables of k_event: matrices, cumulative
// sampling tables (padded, TabLayout<true>) and the azimuth tables
__host__ __device__ inline size_t event_table_doubles(int nmat, bool sym) {
    return (size_t)nmat * ((sym ? TabLayout<true>::MAT4 : TabLayout<true>::MAT) + TabLayout<true>::CUM) + 2 * (NANG + 1);
}
// the same unpadded (k_event TPAD = false: the global layout)
__host__ __device__ inline size_t event_table_doubles_unpadded(int nmat, bool sym) {
    return (size_t)nmat * ((sym ? NANG * 4 : MAT_DOUBLES) + CUM_DOUBLES) + 2 * (NANG + 1);
}
// the same for the cumulative tables and the azimuth tables alone (LDS_C)
__host__ __device__ inline size_t event_cum_doubles(int nmat) {
    return (size_t)nmat * TabLayout<true>::CUM + 2 * (NANG + 1);
}

// peel-off contribution + scattering (ARTES.f90:4765-4984, 819-846).
//  LDS_T: the scattering tables (one 31 KB set per distinct matrix) are staged in LDS --
//         the angle sampling is two binary searches whose every probe depends on the
//         previous one, so each probe's latency (LDS ~100 cycles, L2 ~500) is paid in full.
//  LDS_D: the block accumulates planes 0-8 of the detector in LDS and adds them to its
//         HBM copy once at the end.  Float atomics to HBM execute at the memory side and
//         stay in vmcnt for thousands of cycles, so every later load of the wave waited
//         for them; the grid is one wave of resident blocks, each looping over many events.
// line 0 of the next event's record loaded one event ahead (32 VGPRs); ARTES_EV_PREFETCH=0
// loads it at the event's start (A/B builds)
#ifndef ARTES_EV_PREFETCH
#define ARTES_EV_PREFETCH 1
#endif
static constexpr bool EV_PREFETCH = ARTES_EV_PREFETCH != 0;
#ifndef ARTES_EVENT_WPE
#define ARTES_EVENT_WPE 2
#endif
//  PIX1:  a one-pixel detector: per-lane sums in LDS slots after the tables, reduced over
//         the wave at the end (DetAcc); no LDS detector then.
//  LDS_C: (without LDS_T) the matrices too many for LDS -- the cloudy atmospheres, ~9 per
//         wavelength at 23 KB each -- but their cumulative tables and the azimuth tables
//         (7.2 KB per matrix) staged: the two 4-ary searches, 8 dependent table reads per
//         event, then wait on LDS, and only the interpolation's independent row reads go to
//         L2.  (The call's matrices are its wavelength's only: the host remaps matrix ids
//         per wavelength, transport.hip, wl_set.)
//  ORD:   planes 0-9 as 128-bit fixed-point integers (DetAcc DM_ORD; tuning "det_ordered"):
//         bit-reproducible detector images, no LDS detector or per-lane sums.  1: added to the
//         block's HBM copy at once; 2: accumulated in LDS (integer LDS atomics) and added to the
//         HBM copy at the end of the block (128-bit adds of the block's sums: still exact).
//  TPAD:  (with LDS_T) the tables in LDS padded against bank conflicts (17 / 5 doubles per row) or,
//         when only that fits, unpadded -- the global layout (the cloudy calls' 9 matrices per
//         wavelength: 104 KB unpadded beside the one-pixel lane slots, 130 KB padded)
template <bool LDS_T, bool LDS_D, bool PIX1 = false, int EB = BLOCK, bool LDS_C = false, int ORD = 0, bool TPAD = true>
__global__ __launch_bounds__(EB) __attribute__((amdgpu_waves_per_eu(ARTES_EVENT_WPE, 8))) void k_event(DevGrid G0, DevRun R, Pool S, SubLists SL) {
    static_assert(!(PIX1 && LDS_D), "a one-pixel detector is reduced per lane");
    static_assert(!(ORD && (PIX1 || LDS_D)), "the ordered detector is accumulated in integers");
    constexpr int DM = ORD ? DM_ORD : (PIX1 ? DM_PIX1 : DM_ATOM);
    static_assert(!(LDS_T && LDS_C), "LDS_C stages the cumulative tables alone");
    const Lists L = SL.l[sub_of_block()];
    extern __shared__ double s_ev[];
    DevGrid G = G0;
    const size_t plane = (size_t)R.nx * R.ny;
    double* lds_next = s_ev;
    if constexpr (LDS_C) {
        using TL = TabLayout<true>;
        const int nc = G0.nmat * CUM_DOUBLES;
        double* c = s_ev;
        double* a = c + G0.nmat * TL::CUM;
        double* b = a + (NANG + 1);
        for (int i = threadIdx.x; i < nc; i += EB) {   // entries of 4 -> 5 (cum_at)
            const int e = i >> 2, mm = e / (NANG + 1);
            c[mm * TL::CUM + cum_at<TL::CS>(e - mm * (NANG + 1), i & 3)] = G0.cums[i];
        }
        for (int i = threadIdx.x; i <= NANG; i += EB) { a[i] = G0.sc2[i]; b[i] = G0.ss2[i]; }
        G.cums = c; G.sc2 = a; G.ss2 = b;
        lds_next = b + (NANG + 1);
    }
    if constexpr (LDS_T && !TPAD) {   // the global layout, copied
        const int nm = G0.nmat * (G0.msym ? NANG * 4 : MAT_DOUBLES), nc = G0.nmat * CUM_DOUBLES;
        double* m = s_ev;
        double* c = m + nm;
        double* a = c + nc;
        double* b = a + (NANG + 1);
        for (int i = threadIdx.x; i < nm; i += EB) m[i] = G0.mats[i];
        for (int i = threadIdx.x; i < nc; i += EB) c[i] = G0.cums[i];
        for (int i = threadIdx.x; i <= NANG; i += EB) { a[i] = G0.sc2[i]; b[i] = G0.ss2[i]; }
        G.mats = m; G.cums = c; G.sc2 = a; G.ss2 = b;
        lds_next = b + (NANG + 1);
    }
    if constexpr (LDS_T && TPAD) {
        using TL = TabLayout<true>;
        const int nc = G0.nmat * CUM_DOUBLES;
        double* m = s_ev;
        double* c = m + G0.nmat * (G0.msym ? TL::MAT4 : TL::MAT);
        double* a = c + G0.nmat * TL::CUM;
        double* b = a + (NANG + 1);
        if (G0.msym) {
            for (int i = threadIdx.x; i < G0.nmat * NANG * 4; i += EB) m[(i >> 2) * TL::RS4 + (i & 3)] = G0.mats[i];   // rows of 4 -> 5
        } else {
            for (int i = threadIdx.x; i < G0.nmat * MAT_DOUBLES; i += EB) m[(i >> 4) * TL::RS + (i & 15)] = G0.mats[i];   // rows of 16 -> 17
        }
        for (int i = threadIdx.x; i < nc; i += EB) {   // entries of 4 -> 5 (cum_at)
            const int e = i >> 2, mm = e / (NANG + 1);
            c[mm * TL::CUM + cum_at<TL::CS>(e - mm * (NANG + 1), i & 3)] = G0.cums[i];
        }
        for (int i = threadIdx.x; i <= NANG; i += EB) { a[i] = G0.sc2[i]; b[i] = G0.ss2[i]; }
        G.mats = m; G.cums = c; G.sc2 = a; G.ss2 = b;
        lds_next = b + (NANG + 1);
    }
    double* __restrict__ det = R.det + (size_t)(blockIdx.x % R.ncopy) * R.det_stride;
    double* __restrict__ acc = det;
    if constexpr (LDS_D) {
        acc = lds_next;
        for (size_t i = threadIdx.x; i < 9 * plane; i += EB) acc[i] = 0.0;
    }
    unsigned long long* __restrict__ fix_hbm = ORD ? R.fix + (size_t)(blockIdx.x % R.nfix) * R.fix_stride : nullptr;
    unsigned long long* __restrict__ fix = fix_hbm;
    if constexpr (ORD == 2) {   // the block's fixed-point planes 0-9 in LDS
        fix = (unsigned long long*)lds_next;
        for (size_t i = threadIdx.x; i < 20 * plane; i += EB) fix[i] = 0ull;
    }
    if constexpr (LDS_T || LDS_D || LDS_C || ORD == 2) __syncthreads();
    DetAcc<DM> D;
    D.init(det, acc, plane, lds_next, EB, fix);
    const int n = *L.event_n;
    uint32_t c_scat = 0, c_det = 0;
    const int n_pad = (n + 63) & ~63;   // whole waves iterate together (wave-aggregated appends)
    // Software pipeline: the slot ids come two events ahead and line 0 of the next event's
    // record one event ahead, so the record loads (random lines in the pool) overlap the
    // current event's arithmetic instead of stalling at its start.
    const int stride = sub_grid() * EB;
    int i = sub_block() * EB + threadIdx.x;
    int slot = i < n ? L.event[i] : -1;
    int slot_n = i + stride < n ? L.event[i + stride] : -1;
    Line0 cur;
    if (EV_PREFETCH && slot >= 0) cur = *(const Line0*)(S.s + slot);
#ifdef ARTES_DEBUG_TIMING
    __shared__ unsigned long long s_evtm[EB / 64][32];
    unsigned long long* const ev_tm = s_evtm[threadIdx.x >> 6];
    if ((threadIdx.x & 63) < 32) ev_tm[threadIdx.x & 63] = 0;
    __builtin_amdgcn_wave_barrier();
#endif
    EV_TICK(tl0);
    for (; i < n_pad; i += stride) {
        const int slot_nn = i + 2 * stride < n ? L.event[i + 2 * stride] : -1;
        Line0 nxt;
        if constexpr (EV_PREFETCH) {
            if (slot_n >= 0) nxt = *(const Line0*)(S.s + slot_n);
        } else {
            if (slot >= 0) cur = *(const Line0*)(S.s + slot);
        }
#ifdef ARTES_DEBUG
        if (i < n) dbg_claim(R, L, slot, S.P, 1, slot >= 0 && to_event_list(cur.mode));
#endif
        EV_TICK(te0);
#ifdef ARTES_DEBUG_TIMING
        const int dest = slot >= 0 ? event_one<DM, LDS_T && TPAD, (LDS_T && TPAD) || LDS_C>(G, R, S, slot, cur, D, c_scat, c_det, ev_tm) : 0;
#else
        const int dest = slot >= 0 ? event_one<DM, LDS_T && TPAD, (LDS_T && TPAD) || LDS_C>(G, R, S, slot, cur, D, c_scat, c_det) : 0;
#endif
        EV_TICK(te1);
        EV_ADD(21, te1 - te0);
        EV_ADD(26, 1);
        // the next propagation trace goes to the same position of the output trace list
        // (a hole, -1, for a dropped packet): no list-counter atomic, coalesced stores
#ifdef ARTES_DEBUG
        if (i < n && i >= L.P) atomicAdd(&R.err[ARTES_ERR_LISTS], 1ULL);   // (L2: no write past the list)
        if (i < n && i < L.P) L.trace_out[R.emit_first ? L.P - 1 - i : i] = (dest == 1) ? slot : -1;
#else
        if (i < n) L.trace_out[R.emit_first ? L.P - 1 - i : i] = (dest == 1) ? slot : -1;
#endif
        wave_append(dest == 2, emit_entry(slot, S_END_DROP), L.emit, L.emit_n);   // (event_one set S_END_DROP)
        EV_TICK(te2);
        EV_ADD(25, te2 - te1);
        slot = slot_n;
        slot_n = slot_nn;
        if constexpr (EV_PREFETCH) cur = nxt;
#ifdef ARTES_DEBUG_TIMING
        asm volatile("" ::"v"(cur.px), "v"(cur.mode), "v"(cur.q3), "v"(cur.r0));   // (the copy's wait inside the region)
#endif
        EV_TICK(te3);
        EV_ADD(20, te3 - te2);
    }
    EV_TICK(tl1);
    EV_ADD(27, tl1 - tl0);
#ifdef ARTES_DEBUG_TIMING
    __builtin_amdgcn_wave_barrier();
    if ((threadIdx.x & 63) >= 20 && (threadIdx.x & 63) < 28) atomicAdd(&R.err[threadIdx.x & 63], ev_tm[threadIdx.x & 63]);
#endif
    D.flush_wave();
    if constexpr (ORD == 2) {   // the block's integer sums into its HBM copy, 128 bits each
        __syncthreads();
        for (size_t i = threadIdx.x; i < 10 * plane; i += EB) {
            const unsigned long long lo = fix[2 * i], hi = fix[2 * i + 1];
            if ((lo | hi) == 0) continue;
            const unsigned long long old = atomicAdd(fix_hbm + 2 * i, lo);
            atomicAdd(fix_hbm + 2 * i + 1, hi + (old + lo < old ? 1ull : 0ull));
        }
    }
    if constexpr (LDS_D) {
        __syncthreads();
        for (size_t i = threadIdx.x; i < 9 * plane; i += EB) {
            const double v = acc[i];
            if (v != 0.0) unsafeAtomicAdd(&det[i], v);
        }
    }
    const unsigned long long ws = wave_sum_u64(c_scat), wd = wave_sum_u64(c_det);
    if ((threadIdx.x & 63) == 0) {
        if (ws) cnt_add(R, ARTES_CNT_SCATTERS, ws);
        if (wd) cnt_add(R, ARTES_CNT_DETECTED, wd);
    }
}

// emit_photon, planet branch (ARTES.f90:1117-1266): a cell drawn from the emissivity CDF
// (a binary search finds the entry the reference's linear scan stops at, 1126-1154), a
// uniform point in it, and an isotropic or upward-biased direction
__device__ __forceinline__ void emit_planet(const DevGrid& G, const DevRun& R, Rng& rng, double& px, double& py, double& pz,
                                            double& dx, double& dy, double& dz, int& cr, int& ct, int& cp, double& bias) {
    bias = 1.0;
    const double samp = rng.uni() * G.th_total;
    int lo = 0, hi = G.th_ncdf - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (G.th_cdf[mid] >= samp) hi = mid;
        else lo = mid + 1;
    }
    const int per_r = G.ntheta * G.nphi;
    cr = G.th_cd0 + lo / per_r; ct = (lo / G.nphi) % G.ntheta; cp = lo % G.nphi;
    const double r = G.rfr[cr] + rng.uni() * (G.rfr[cr + 1] - G.rfr[cr]);
    const double ctheta = G.tcos[ct] + rng.uni() * (G.tcos[ct + 1] - G.tcos[ct]);
    const double stheta = sqrt(1.0 - ctheta * ctheta);
    double ph;
    const double xi = rng.uni();
    if (G.nphi == 1) ph = TWO_PI * xi;
    else if (cp < G.nphi - 1) ph = G.phif[cp] + xi * (G.phif[cp + 1] - G.phif[cp]);
    else ph = G.phif[cp] + xi * (TWO_PI - G.phif[cp]);
    const double cph = cos_b(ph);
    double sph = sqrt(1.0 - cph * cph);
    if (ph > PI) sph = -sph;
    px = G.ox * (r * stheta * cph);
    py = G.oy * (r * stheta * sph);
    pz = G.oz * (r * ctheta);
    if (R.photon_emission == 2) {   // biased upward (Gordon 1987), ARTES.f90:1233-1254
        const double b = R.photon_bias;
        const double yb = (1.0 + b) * tan(PI * rng.uni() / 2.0) / sqrt(1.0 - b * b);
        const double ths = acos((1.0 - yb * yb) / (1.0 + yb * yb));
        const double beta = TWO_PI * rng.uni();
        double n0, n1, n2;
        surface_normal(G, px, py, pz, n0, n1, n2);
        direction_cosine(R, cos_b(PI - ths), beta, n0, n1, n2, dx, dy, dz);
        bias = (PI * sin_b(ths) * (1.0 + b * cos_b(ths))) / (2.0 * sqrt(1.0 - b * b));
    } else {                        // isotropic, ARTES.f90:1218-1231
        const double alpha = 2.0 * rng.uni() - 1.0;
        const double beta = TWO_PI * rng.uni();
        const double cb = cos_b(beta);
        double sb = sqrt(1.0 - cb * cb);
        if (beta > PI) sb = -sb;
        dx = sqrt(1.0 - alpha * alpha) * cb;
        dy = sqrt(1.0 - alpha * alpha) * sb;
        dz = alpha;
    }
    if (fabs(dz) >= 1.0) log_err(R, 54);
}

// close finished packets and emit new ones (ARTES.f90:546-597, 1027-1115, 2605-2669)
//
// Emit-list entry i takes packet id next_pkt + i (ids < n only) and writes its new trace
// to position out0 + i of the output trace list (see Lists), a hole (-1)
// when the ids have run out: list positions and packet ids need no atomics, and the
// packet-to-slot assignment is deterministic.  k_rotate advances next_pkt and the count.
// doubles of LDS k_emit stages for initial_cell: keys and faces of theta [ntheta+1] and phi [nphi] + 1
__host__ __device__ inline size_t emit_table_doubles(int ntheta, int nphi) { return 2 * ((size_t)ntheta + 1 + nphi + 1); }

// the cell j of ascending faces f[0..n] with f[j] < v < f[j+1], or 0 when v sits on a face
// or outside: the cell initial_cell's linear scan finds (ARTES.f90:2630-2660).  Binary
// search: the scan's dependent loads were most of k_emit's time
__device__ __forceinline__ int face_interval(const double* f, int n, double v) {
    int lo = 0, hi = n - 1, j = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (f[mid] < v) { j = mid; lo = mid + 1; }
        else hi = mid - 1;
    }
    return (j >= 0 && v < f[j + 1]) ? j : 0;
}

// face_interval over an increasing key of the angle (k_emit's initial_cell): the same cell as
// the search over the angle itself whenever the key lies 1e-9 or more from both bounding
// faces' keys (the keys below grow no faster than their angle, so the angle is then 1e-9 rad
// or more from the faces, far beyond the rounding of acos / atan2); `near` otherwise (or NaN)
__device__ __forceinline__ int key_interval(const double* f, int n, double v, bool& near) {
    int lo = 0, hi = n - 1, j = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (f[mid] < v) { j = mid; lo = mid + 1; }
        else hi = mid - 1;
    }
    const int jj = j < 0 ? 0 : j;
    near = !(v - f[jj] >= 1.e-9 && f[jj + 1] - v >= 1.e-9);
    return jj;
}

// a key of the angle atan2(y, x) in [0, 2 pi) that grows with it, in [0, 4): one unit per
// quadrant, a ratio of |x| or |y| to |x| + |y| (no atan2).  d key / d angle = 1 / (|cos| +
// |sin|)^2, in [1/2, 1]
__device__ __forceinline__ double phi_key(double x, double y) {
    const double ax = fabs(x), ay = fabs(y), q = 1.0 / (ax + ay);
    if (!(y < 0.0)) return x >= 0.0 ? ay * q : 1.0 + ax * q;
    return x < 0.0 ? 2.0 + ay * q : 3.0 + ax * q;
}

// Store every lane's 128-byte line, staged in LDS at st[9 * lane ...], to `dst` (null:
// none), the whole wave together (wave-uniform control flow): groups of 8 lanes write 16
// bytes each, so every store instruction writes 8 whole lines.  Written per lane, each of
// the 8 instructions would touch 64 lines, one 16-byte piece of each.
constexpr int LINE_STAGE = 64 * 9;   // uint4 per wave: 64 lines of 8 pieces, padded to 9
__device__ __forceinline__ void wave_store_lines(const uint4* st, void* dst) {
    const int l = threadIdx.x & 63;
    __builtin_amdgcn_wave_barrier();
    const unsigned long long d = (unsigned long long)dst;
    const int lo = (int)(unsigned)d, hi = (int)(d >> 32);
    const int piece = l & 7;
#pragma unroll 1
    for (int r = 0; r < 8; r++) {
        const int src = r * 8 + (l >> 3);
        const unsigned long long a = ((unsigned long long)(unsigned)__shfl(hi, src) << 32) | (unsigned)__shfl(lo, src);
        if (a) reinterpret_cast<uint4*>(a)[piece] = st[src * 9 + piece];
    }
    __builtin_amdgcn_wave_barrier();
}

// STAR: the star source alone (photon:source=star) -- no thermal emission, no flux sums -- so the
// planet branch's registers do not set the kernel's budget: 106 VGPRs on 3D grids (159 with the
// branch), 4 waves per SIMD instead of 3 (the LDS line stage allows 4 blocks per CU).  k_emit
// waits on memory; the 4th wave hides more of it: bench k_emit 38.9 -> 34.3 ms per step
// (profiles/r06/ab/emit_star_waves_ab.txt; radial-only grids: 98 VGPRs either way, no hint)
template <bool G3D, bool TRACE, bool STAR = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu((STAR && G3D) ? 4 : 1))) void k_emit(DevGrid G, DevRun R, Pool S, SubLists SL) {
    const Lists L = SL.l[sub_of_block()];
    extern __shared__ double s_em[];
    __shared__ uint4 s_lines[BLOCK / 64 * LINE_STAGE];
    // initial_cell's searches, over keys of the angles: -cos(theta) of the theta faces, phi_key
    // of the phi faces (then 4); the faces themselves for the rare position near a face
    double* s_tk = s_em;                          // [ntheta + 1]
    double* s_pk = s_tk + (G.ntheta + 1);         // [nphi + 1]
    double* s_tf = s_pk + (G.nphi + 1);           // [ntheta + 1]
    double* s_pf = s_tf + (G.ntheta + 1);         // [nphi + 1]: the faces, then 2 pi
    if constexpr (G3D) {
        for (int i = threadIdx.x; i <= G.ntheta; i += BLOCK) {
            s_tk[i] = -G.tcos[i];
            s_tf[i] = G.thetaf[i];
        }
        for (int i = threadIdx.x; i < G.nphi; i += BLOCK) {
            s_pk[i] = phi_key(G.phic[i], G.phis[i]);
            s_pf[i] = G.phif[i];
        }
        if (threadIdx.x == 0) {
            s_pk[G.nphi] = 4.0;
            s_pf[G.nphi] = TWO_PI;
        }
        __syncthreads();
    }
    const int n = *L.emit_n;
    const int out0 = R.emit_first ? 0 : *L.event_n;
    const unsigned long long pkt0 = *L.next_pkt;
    const size_t plane = (size_t)R.nx * R.ny;
    double* __restrict__ det = R.det + (size_t)(blockIdx.x % R.ncopy) * R.det_stride;
    uint32_t c_exit = 0, c_abs = 0, c_drop = 0, c_pkt = 0;
    double t2[4] = {0, 0, 0, 0};
    double f_emit = 0.0, f_exit = 0.0;   // thermal flux_emitted / flux_exit (ARTES.f90:607, 780, 953)
    const int n_pad = (n + 63) & ~63;
    for (int i = sub_block() * BLOCK + threadIdx.x; i < n_pad; i += sub_grid() * BLOCK) {
        const int e = i < n ? L.emit[i] : -1;
        const int slot = e >= 0 ? (e & 0x07FFFFFF) : -1, code = e >= 0 ? (e >> 27) & 3 : 0;
        // (code 0 is a fresh slot, (L3): its record is not read -- k_init leaves it unwritten
        // outside the debug build, and this kernel writes the whole line before any use)
#ifdef ARTES_DEBUG
        const int m = code ? S_END_EXIT - 1 + code : (slot >= 0 ? S.s[slot].mode : S_RETIRED);
#else
        const int m = code ? S_END_EXIT - 1 + code : (slot >= 0 ? (int)S_FRESH : (int)S_RETIRED);
#endif
#ifdef ARTES_DEBUG
        if (i < n) dbg_claim(R, L, slot, S.P, 2, (m == S_END_EXIT || m == S_END_ABS || m == S_END_DROP || m == S_FRESH) &&
                                                     (slot < 0 || S.s[slot].mode == m));
#endif
        if (m == S_END_EXIT || m == S_END_ABS || m == S_END_DROP) {
            if (m == S_END_EXIT) c_exit++;
            else if (m == S_END_ABS) c_abs++;
            else c_drop++;
            if (R.moments) {
                const int cur = S.d[slot].cur_pix;
                if (cur >= 0) {
                    unsafeAtomicAdd(&det[12 * plane + cur], S.d[slot].cs0 * S.d[slot].cs0);
                    unsafeAtomicAdd(&det[13 * plane + cur], S.d[slot].cs1 * S.d[slot].cs1);
                    unsafeAtomicAdd(&det[14 * plane + cur], S.d[slot].cs2 * S.d[slot].cs2);
                    unsafeAtomicAdd(&det[15 * plane + cur], S.d[slot].cs3 * S.d[slot].cs3);
                }
                const double a0 = S.d[slot].pt0, a1 = S.d[slot].pt1, a2 = S.d[slot].pt2, a3 = S.d[slot].pt3;
                t2[0] += a0 * a0; t2[1] += a1 * a1; t2[2] += a2 * a2; t2[3] += a3 * a3;
            }
            if (!STAR && m == S_END_EXIT && R.photon_source == 2) f_exit += S.s[slot].wI;
            if constexpr (TRACE) {
                double* rr = R.rec + (size_t)(S.d[slot].pid - R.first) * ARTES_TRACE_FIELDS;
                rr[0] = S.d[slot].peel_sum;
                rr[1] = (double)S.d[slot].nscat;
                rr[2] = (double)S.s[slot].ncross;
                rr[3] = (double)(m - S_END_EXIT + 1);   // 1 exit, 2 absorbed, 3 dropped
                rr[4] = S.d[slot].peel_pol[0];
                rr[5] = S.d[slot].peel_pol[1];
                rr[6] = S.d[slot].peel_pol[2];
                rr[7] = 0.0;
            }
        }
        const unsigned long long k = pkt0 + (unsigned long long)i;
        const bool emit = slot >= 0 && k < L.n;
        if (slot >= 0 && !emit) S.s[slot].mode = S_RETIRED;
        uint4* const st = s_lines + (threadIdx.x >> 6) * LINE_STAGE;
        Line0& rec = *reinterpret_cast<Line0*>(st + (threadIdx.x & 63) * 9);   // (stored below by the whole wave)
        if (emit) {
        c_pkt++;
        const unsigned long long pid = L.first + k;
        Rng rng;
        rng.seed(R.seed, pid);
        double px, py, pz, dx, dy, dz, wI = 1.0;
        int cr = G.nr - 1, ct = 0, cp = 0, face = pack_face(1, G.nr), mode0 = S_FIRST;
        if (!STAR && R.photon_source == 2) {
            double bias;
            emit_planet(G, R, rng, px, py, pz, dx, dy, dz, cr, ct, cp, bias);
            // weight for the cell emission probability (ARTES.f90:605), then peel_thermal
            wI = bias / G.th_weight[cr + G.nr * (ct + G.ntheta * cp)];
            f_emit += wI;
            face = pack_face(0, 0);
            mode0 = S_PEEL_T;
        } else {
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
        double sphi, cphi;
        sincos_bounded(phi_disk, sphi, cphi);
        const double d1 = Rt * r_disk * sphi, d2 = Rt * r_disk * cphi;
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
        if constexpr (G3D) {   // initial_cell (ARTES.f90:2605-2669)
            // (the searches over keys of the angles; acos / atan2 only near a face, ~1e-7 of the
            // packets: they were ~30 % of k_emit's instructions)
            const double r = sqrt(px * px + py * py + pz * pz);
            bool near_t, near_p;
            ct = key_interval(s_tk, G.ntheta, -(pz / r), near_t);
            cp = key_interval(s_pk, G.nphi, phi_key(px, py), near_p);
            if (near_t) ct = face_interval(s_tf, G.ntheta, acos(pz / r));
            if (near_p) {
                double ph = atan2(py, px);
                if (ph < 0.0) ph += TWO_PI;
                cp = face_interval(s_pf, G.nphi, ph);
            }
        }
        }   // star
        rec.r0 = rng.s0; rec.r1 = rng.s1;
        rec.px = px; rec.py = py; rec.pz = pz;
        rec.dx = dx; rec.dy = dy; rec.dz = dz;
        rec.q1 = 0.0; rec.q2 = 0.0; rec.q3 = 0.0;
        rec.wI = wI;
        rec.pcell = pack_cell(cr, ct, cp); rec.pface = face;
        rec.ttgt = 0.0;
        rec.tpeel = 0.0;
        rec.ncross = 0;
        rec.mode = mode0;
        if (R.moments) {
            S.d[slot].cs0 = S.d[slot].cs1 = S.d[slot].cs2 = S.d[slot].cs3 = 0.0;
            S.d[slot].pt0 = S.d[slot].pt1 = S.d[slot].pt2 = S.d[slot].pt3 = 0.0;
            S.d[slot].cur_pix = -1;
        }
        if constexpr (TRACE) {
            S.d[slot].pid = pid;
            S.d[slot].peel_sum = 0.0;
            S.d[slot].peel_pol[0] = S.d[slot].peel_pol[1] = S.d[slot].peel_pol[2] = 0.0;
            S.d[slot].nscat = 0;
        }
        }   // emit
        wave_store_lines(st, emit ? (void*)&S.s[slot] : nullptr);
#ifdef ARTES_DEBUG
        if (i < n && out0 + i >= L.P) atomicAdd(&R.err[ARTES_ERR_LISTS], 1ULL);   // (L2: no write past the list)
        if (i < n && out0 + i < L.P) L.trace_out[out0 + i] = emit ? slot : -1;
#else
        if (i < n) L.trace_out[out0 + i] = emit ? slot : -1;
#endif
    }
    const unsigned long long a = wave_sum_u64(c_exit), b = wave_sum_u64(c_abs), c = wave_sum_u64(c_drop),
                             d = wave_sum_u64(c_pkt);
    const double q0 = wave_sum_f64(t2[0]), q1 = wave_sum_f64(t2[1]), q2 = wave_sum_f64(t2[2]), q3 = wave_sum_f64(t2[3]);
    if ((threadIdx.x & 63) == 0) {
        if (a) cnt_add(R, ARTES_CNT_EXITED, a);
        if (b) cnt_add(R, ARTES_CNT_ABSORBED, b);
        if (c) cnt_add(R, ARTES_CNT_DROPPED, c);
        if (d) cnt_add(R, ARTES_CNT_PACKETS, d);
        if (q0 != 0.0) tot_add(R, 0, q0);
        if (q1 != 0.0) tot_add(R, 1, q1);
        if (q2 != 0.0) tot_add(R, 2, q2);
        if (q3 != 0.0) tot_add(R, 3, q3);
    }
    if (!STAR && R.photon_source == 2) {
        const double fe = wave_sum_f64(f_emit), fx = wave_sum_f64(f_exit);
        if ((threadIdx.x & 63) == 0) {
            if (fe != 0.0) tot_add(R, 4, fe);
            if (fx != 0.0) tot_add(R, 5, fx);
        }
    }
}

// initial fill: the first `use` slots are fresh and queued for emission (a run of fewer
// packets than the pool holds leaves the rest untouched: no list ever names them)
// the first `use[s]` slots of every sub-engine s are free and queued for emission
struct SubUse {
    int u[NSUB];
};
__global__ void k_init(Pool S, int* emit, int* emit_n /*[NSUB], CPAD apart*/, int Ps, SubUse use) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Ps * NSUB) return;
    const int sub = i / Ps, j = i - sub * Ps;
    if (j < use.u[sub]) {
#ifdef ARTES_DEBUG
        S.s[i].mode = S_FRESH;   // (only the debug build's list checks read a fresh slot's mode)
#endif
        emit[i] = i;   // position j of sub-engine sub's emit list
    }
    if (j == 0) emit_n[sub * CPAD] = use.u[sub];
}

// end of an iteration: the output trace list (k_event's event_n entries, then k_emit's
// emit_n) becomes the input, the consumed input buffer is reset to become the next
// output, packet ids advance by the emit-list length; event/emit lists and cursors are zeroed
// (one block per sub-engine; counters are laid out [field][NSUB], CPAD ints apart: cnt_at)
enum : int { CNT_IN0 = 0, CNT_IN1 = 1, CNT_EVENT = 2, CNT_EMIT = 3, CNT_SPLIT0 = 4, CNT_SPLIT1 = 5, CNT_DBG = 8, CNT_FIELDS = 16 };
__host__ __device__ constexpr int cnt_at(int field, int sub) { return (field * NSUB + sub) * CPAD; }
__global__ void k_rotate(int* cnt, int in, unsigned int* grab_all, unsigned long long* next_all, int emit_first, int P,
                         unsigned long long* err) {
    const int sub = blockIdx.x;
    int* in_n = cnt + cnt_at(CNT_IN0 + in, sub);
    int* out_n = cnt + cnt_at(CNT_IN0 + 1 - in, sub);
    int* out_split = cnt + cnt_at(CNT_SPLIT0 + 1 - in, sub);
    int* event_n = cnt + cnt_at(CNT_EVENT, sub);
    int* emit_n = cnt + cnt_at(CNT_EMIT, sub);
    int* dbg_iter = cnt + cnt_at(CNT_DBG, sub);
    unsigned int* grab = grab_all + grab_at(sub, 0);
    unsigned long long* next_pkt = next_all + sub;
    (void)dbg_iter; (void)err;
    if (threadIdx.x == 0) {
        const int ev = *event_n, em = *emit_n;
#ifdef ARTES_DEBUG
        if (ev < 0 || em < 0 || ev + em > P) atomicAdd(&err[ARTES_ERR_LISTS], 1ULL);   // (L2)
        *dbg_iter += 1;
#endif
        *out_n = ev + em;
        *out_split = emit_first ? em : ev + em;
        *next_pkt += (unsigned long long)em;
        *in_n = 0;
        *event_n = 0;
        *emit_n = 0;
    }
    if (threadIdx.x < 8) grab[threadIdx.x * CPAD] = 0;
}

}  // namespace artes
