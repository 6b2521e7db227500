// orbit_post.hip — MI355X (gfx950) kernels for SURVEY.md §8(f) rows f3 and f4, the
// consumer and the producer either side of the orbit-tagging path, behind the C ABI
// of include/orbit_post.h (second translation unit of liborbit_hip.so).
//
// Reference (paths under /root/reference/orbitanalysis/):
//   Apsides.collate_apsides        postprocessing.py:118-142 -> k_collate_rank,
//                                  k_collate_offsets, k_collate_place
//   Apsides.save_final_apsis_counts postprocessing.py:215-236 -> k_retro_counts
//   get_central_particle_ids       progenitors.py:38-56       -> k_central
//   find_main_progenitors          progenitors.py:82-117      -> k_mp_insert,
//                                  k_mp_probe, k_mp_lookup, k_mp_tally
//
// Design: no global sort anywhere.
//  * collate keeps, per collated halo, the cumulative sorted-unique (ID, count) list
//    the reference rebuilds with np.unique every snapshot; a snapshot's kept apsis IDs
//    are sorted per halo in LDS (bitonic, <= OA_COLLATE_CHUNK keys) and run-length
//    encoded, the old list streams past them (binary search in LDS) to count the
//    merged length; after a scan of the lengths a second per-halo pass writes every
//    element at its merge rank;
//  * central IDs: per region block, an MSB-first radix select of the n-th smallest
//    radius (common high bits skipped, early exit when a bin is taken whole; keys
//    cached in LDS for blocks <= 12288) and an LDS bitonic sort of the <= n
//    survivors by (radius, position);
//  * main progenitors: an open-addressing table over the tracked IDs (first
//    occurrence) behind an L2-resident bit filter; the halo members are streamed past
//    it once, then a per-block LDS tally.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <math.h>

#include "orbit_hip.h"
#include "orbit_post.h"

void oa_internal_error(const char *msg);   // orbit_hip.hip: owns oa_last_error()'s buffer

namespace {

int fail(int code, const char *msg) {
    oa_internal_error(msg);
    return code;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) return OA_OK;
    char b[256];
    snprintf(b, sizeof(b), "%s: %s", what, hipGetErrorString(e));
    return fail(OA_E_LAUNCH, b);
}

constexpr uint64_t SIGN = 0x8000000000000000ull;
constexpr int CH = OA_COLLATE_CHUNK;
constexpr int SC = OA_CENTRAL_MAX_N;     // k_central: survivors sorted in LDS

#ifndef OA_STAMPS
#define OA_STAMPS 0
#endif
#if OA_STAMPS
// diagnostic builds: per-block s_memrealtime at the phase boundaries of k_central
// (OA_STAMPS=1) or k_collate_rank (OA_STAMPS=2)
constexpr int CST_N = 8, CST_MAX = 1 << 16;
__device__ uint64_t g_cstamps[CST_MAX * CST_N];
#define STAMP_AT(k) do { if (threadIdx.x == 0 && blockIdx.x < CST_MAX) \
    g_cstamps[blockIdx.x * CST_N + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#endif
#if OA_STAMPS == 1
#define CSTAMP(k) STAMP_AT(k)
#else
#define CSTAMP(k) do { } while (0)
#endif
#if OA_STAMPS == 2
#define RSTAMP(k) STAMP_AT(k)
#else
#define RSTAMP(k) do { } while (0)
#endif

// value of element i as 64-bit two's complement (signed kinds sign-extend)
__device__ __forceinline__ uint64_t load_val(const void *p, int64_t i, int kind) {
    switch (kind) {
        case OA_ID_I64:
        case OA_ID_U64: return static_cast<const uint64_t *>(p)[i];
        case OA_ID_I32: return (uint64_t)(int64_t) static_cast<const int32_t *>(p)[i];
        default: return (uint64_t) static_cast<const uint32_t *>(p)[i];
    }
}
// streamed-once IDs (non-temporal: L2 stays with the tables and filters read at random)
template <int KIND> __device__ __forceinline__ uint64_t load_val_nt(const void *p, int64_t i) {
    if constexpr (KIND == OA_ID_I64 || KIND == OA_ID_U64)
        return __builtin_nontemporal_load(static_cast<const uint64_t *>(p) + i);
    else if constexpr (KIND == OA_ID_I32)
        return (uint64_t)(int64_t)__builtin_nontemporal_load(static_cast<const int32_t *>(p) + i);
    else
        return (uint64_t)__builtin_nontemporal_load(static_cast<const uint32_t *>(p) + i);
}
__device__ __forceinline__ uint64_t to_key(uint64_t v, int key_signed) {
    return key_signed ? v ^ SIGN : v;
}
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xFF51AFD7ED558CCDull; x ^= x >> 33; x *= 0xC4CEB9FE1A85EC53ull;
    return x ^ (x >> 33);
}
// largest j in [0, n) with off[j] <= t  (the segment holding t; empty segments precede it)
__device__ __forceinline__ int seg_of(const int64_t *off, int n, int64_t t) {
    int lo = 0, hi = n;                  // invariant: off[lo] <= t (callers guarantee off[0] <= t)
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (off[mid] <= t) lo = mid; else hi = mid;
    }
    return lo;
}

// exclusive work-group scan of one value per thread (NT threads, whole waves)
template <int NT, typename T>
__device__ __forceinline__ T block_scan(T v, T *wsum, T &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    T incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        T acc = 0;
        for (int k = 0; k < NT / 64; ++k) { const T t = wsum[k]; wsum[k] = acc; acc += t; }
        wsum[NT / 64] = acc;
    }
    __syncthreads();
    const T r = wsum[w] + incl - v;
    total = wsum[NT / 64];
    __syncthreads();
    return r;
}

// ascending bitonic sort of P (power of two) keys in LDS, NT threads
template <int NT>
__device__ void bitonic_keys(uint64_t *s, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += NT) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = s[i], b = s[ixj];
                    if ((a > b) == ((i & k) == 0)) { s[i] = b; s[ixj] = a; }
                }
            }
            __syncthreads();
        }
    }
}
// ... of (key, index) pairs, lexicographic
template <int NT>
__device__ void bitonic_pairs(uint64_t *s, uint32_t *x, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += NT) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = s[i], b = s[ixj];
                    const uint32_t ia = x[i], ib = x[ixj];
                    const bool gt = a > b || (a == b && ia > ib);
                    if (gt == ((i & k) == 0)) { s[i] = b; s[ixj] = a; x[i] = ib; x[ixj] = ia; }
                }
            }
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------------ f3: collate
// Apsides.collate_apsides (postprocessing.py:118-142) as three launches per round:
//   k_collate_rank   one 256-thread work-group per halo: this round's kept apsis IDs
//                    (angle > cut via the NumPy-evaluated LUT, :127-128) sorted in LDS
//                    and run-length encoded (np.unique(return_counts), :135) into u unique
//                    new keys; the halo's old keys stream past them once (binary search
//                    in LDS), giving per new key q: F(q) = #new keys below q already in the
//                    old list, H(q) = #old keys below q; and the merged length
//                    on + u - F(u)  (np.append + np.unique, :130-136);
//   k_collate_offsets  the merged lengths -> offsets (one work-group);
//   k_collate_place  one work-group per halo: old element i (rank L among the new keys)
//                    goes to i + L - F(L), adding the new count when it is new key L;
//                    absent new key q goes to H(q) + q - F(q).
// No cross-work-group waits (a single-pass variant placing halos behind a decoupled
// look-back waited on its slowest predecessors: profiles/r05/ab_collate_lookback_r05su.txt).
constexpr int CT = 256, CL_U = 4;
#ifndef OA_PLACE_MU
#define OA_PLACE_MU 16         // k_collate_place: old elements per thread per trip
#endif

__device__ __forceinline__ int lower_rank(const uint64_t *nk, int u, uint64_t key) {
    int L = 0, R = u;
    while (L < R) {
        const int mid = (L + R) >> 1;
        if (nk[mid] < key) L = mid + 1; else R = mid;
    }
    return L;
}

// KIND: the apsis ID kind (a template argument: the loads below are unconditional, index
// clamped, so CL_U of them are in flight per thread; a load under a lane test or a kind
// switch waits for its data before the next one issues)
#ifndef OA_CTILE_WAVES
#define OA_CTILE_WAVES 2        // k_collate_rank: old keys per LDS tile, in units of CT
#endif
constexpr int CTILE = OA_CTILE_WAVES * CT;

// ascending bitonic sort of the first P (a power of two) keys, held K per thread
// (thread t: keys K t .. K t + K - 1; the threads past P / K idle): a stage whose partner
// is in the same thread swaps registers, one in another lane of the wave exchanges
// through a lane shuffle, one in another wave (j >= 64 K: P > 512 only) through LDS
// (lds: P keys).
template <int K>
__device__ void bitonic_regs(uint64_t (&v)[K], int P, uint64_t *lds) {
    const int t = threadIdx.x;
    const bool active = K * (t & ~63) < P;                   // uniform per wave
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j >= K; j >>= 1) {
            if (j >= 64 * K) {
                if (active)
#pragma unroll
                    for (int r = 0; r < K; ++r) lds[K * t + r] = v[r];
                __syncthreads();
                if (active)
#pragma unroll
                    for (int r = 0; r < K; ++r) {
                        const int i = K * t + r;
                        const uint64_t w = lds[i ^ j];
                        const bool up = (i & k) == 0, lower = (i & j) == 0;
                        v[r] = (up == lower) ? (v[r] < w ? v[r] : w) : (v[r] < w ? w : v[r]);
                    }
                __syncthreads();
            } else if (active) {
                const int mk = j / K;
                const bool lower = (t & mk) == 0;
#pragma unroll
                for (int r = 0; r < K; ++r) {
                    const uint64_t w = __shfl_xor((unsigned long long)v[r], mk);
                    const bool up = ((K * t + r) & k) == 0;
                    v[r] = (up == lower) ? (v[r] < w ? v[r] : w) : (v[r] < w ? w : v[r]);
                }
            }
        }
        if (active)
#pragma unroll
            for (int jj = K / 2; jj > 0; jj >>= 1) {
                if (jj >= k) continue;
#pragma unroll
                for (int r = 0; r < K; ++r) {
                    if (r & jj) continue;
                    const bool up = ((K * t + r) & k) == 0;
                    const uint64_t x = v[r], y = v[r | jj];
                    if ((x > y) == up) { v[r] = y; v[r | jj] = x; }
                }
            }
    }
}

// K: sort keys per thread (lds_keys / CT, at least 2)
// LDS (a.lds_keys = S): [S] u64 sort slots, then the unique new keys in place;
// [max(S + 1, 2 * CTILE)] int run heads, then old-key tiles of CTILE; [S + 1] int flags.
template <int KIND, int K>
__global__ __launch_bounds__(CT) void k_collate_rank(const oa_collate_args a) {
    extern __shared__ __attribute__((aligned(16))) char cl_smem[];
    const int S = a.lds_keys;
    const int hs = S + 1 > 2 * CTILE ? S + 1 : 2 * CTILE;
    uint64_t *sk = reinterpret_cast<uint64_t *>(cl_smem);   // sort slots -> unique new keys
    int *hp = reinterpret_cast<int *>(sk + S);               // run heads -> old-key tiles
    uint64_t *tile = reinterpret_cast<uint64_t *>(hp);
    int *fp = hp + hs;                                       // bit 0: found in the old list,
                                                             // bit 1: lower bound written
    __shared__ int wsum[CT / 64 + 1];
    __shared__ int s_m;
    const int j = blockIdx.x;
    RSTAMP(0);
    const int64_t ob = a.old_off[j], on = a.old_off[j + 1] - ob;
    const int64_t rem = a.src_cnt[j] - a.chunk_start;
    const int nraw = rem <= 0 ? 0 : (rem < CH ? (int)rem : CH);
    const int64_t base = a.new_base[j];
    // the halo's workspace rows [base, base + nraw) must lie in [0, n_new_cap): the w_*
    // stores below are then in bounds (u <= m <= nraw); otherwise report, store nothing
    const bool bad = nraw > 0 && (base < 0 || base + nraw > a.n_new_cap || nraw > a.lds_keys);
    if (nraw == 0 || bad) {                                  // nothing new: the list is kept
        if (threadIdx.x == 0) {
            a.w_ulen[j] = 0; a.w_found[j] = 0;
            if (bad && a.status) atomicOr(a.status, (int32_t)OA_POST_BOUNDS);
        }
        return;
    }
    // the first old-key tile: loads issued now, staged after the sort
    uint64_t okey[CTILE / CT];
    if (on > 0)
#pragma unroll
        for (int e = 0; e < CTILE / CT; ++e) {
            const int64_t i = e * CT + threadIdx.x, ic = i < on ? i : on - 1;
            okey[e] = __builtin_nontemporal_load(a.old_keys + ob + ic);
        }
    if (threadIdx.x == 0) s_m = 0;
    __syncthreads();
    const int64_t s0 = a.src_off[j] + a.chunk_start;
    for (int i0 = 0; i0 < nraw; i0 += CL_U * CT) {
        uint16_t an[CL_U];
        uint64_t id[CL_U];
#pragma unroll
        for (int e = 0; e < CL_U; ++e) {
            const int i = i0 + e * CT + (int)threadIdx.x;
            const int64_t r = s0 + (i < nraw ? i : nraw - 1);
            an[e] = a.angles[r];
            id[e] = load_val_nt<KIND>(a.apsis_ids, r);
        }
        uint8_t kp[CL_U];
#pragma unroll
        for (int e = 0; e < CL_U; ++e) kp[e] = a.keep_lut[an[e]];
#pragma unroll
        for (int e = 0; e < CL_U; ++e) {
            const int i = i0 + e * CT + (int)threadIdx.x;
            // compaction: one LDS atomic per wave, lanes placed by their ballot rank
            const bool keep = i < nraw && kp[e];
            const uint64_t bal = __ballot(keep);
            const int lane = threadIdx.x & 63;
            int wb = 0;
            if (lane == 0 && bal) wb = atomicAdd(&s_m, __popcll(bal));
            wb = __shfl(wb, 0);
            if (keep) sk[wb + __popcll(bal & ((1ull << lane) - 1))] = to_key(id[e], a.key_signed);
        }
    }
    __syncthreads();
    RSTAMP(1);
    const int m = s_m;
    if (m == 0) {
        if (threadIdx.x == 0) { a.w_ulen[j] = 0; a.w_found[j] = 0; }
        return;
    }
    int P = 1;
    while (P < m) P <<= 1;
    {   // sort in registers: thread t holds keys [K t, K t + K), padded with ~0 (ties with a
        // real ~0 key are harmless)
        uint64_t v[K];
        const bool mine = K * (int)threadIdx.x < P;
#pragma unroll
        for (int r = 0; r < K; ++r) {
            const int i = K * (int)threadIdx.x + r;
            v[r] = i < m ? sk[i] : ~0ull;
        }
        __syncthreads();
        bitonic_regs<K>(v, P, sk);
        if (mine)
#pragma unroll
            for (int r = 0; r < K; ++r) sk[K * threadIdx.x + r] = v[r];
        __syncthreads();
    }
    RSTAMP(2);
    int u;
    {   // run heads: thread t owns positions [t*E, t*E + E)
        const int E = (m + CT - 1) / CT;
        const int lo = threadIdx.x * E, hi = min(lo + E, m);
        int nh = 0;
        for (int i = lo; i < hi; ++i) nh += (i == 0 || sk[i] != sk[i - 1]);
        int q = block_scan<CT, int>(nh, wsum, u);
        for (int i = lo; i < hi; ++i)
            if (i == 0 || sk[i] != sk[i - 1]) hp[q++] = i;
        if (threadIdx.x == 0) hp[u] = m;
        __syncthreads();
        // the unique keys move down in place (all read before any is written); their
        // multiplicities go out now, which frees the run heads for the tiles
        uint64_t kq[K];
#pragma unroll
        for (int r = 0; r < K; ++r) {
            const int qq = r * CT + (int)threadIdx.x;
            if (qq < u) {
                kq[r] = sk[hp[qq]];
                a.w_cnt[base + qq] = hp[qq + 1] - hp[qq];
                fp[qq] = 0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < K; ++r) {
            const int qq = r * CT + (int)threadIdx.x;
            if (qq < u) sk[qq] = kq[r];
        }
    }
    __syncthreads();
    RSTAMP(3);
    const uint64_t *nk = sk;
    // lower bound of every new key in the old list: the old keys pass through LDS one
    // tile at a time (the next tile's loads in flight); a key is searched in the tile
    // whose key range holds it
    uint64_t prev_last = 0;
    for (int64_t t0 = 0; t0 < on; t0 += CTILE) {
        const int nt = on - t0 < CTILE ? (int)(on - t0) : CTILE;
#pragma unroll
        for (int e = 0; e < CTILE / CT; ++e) {
            const int i = e * CT + (int)threadIdx.x;
            if (i < nt) tile[i] = okey[e];
        }
        if (t0 + CTILE < on)
#pragma unroll
            for (int e = 0; e < CTILE / CT; ++e) {
                const int64_t i = t0 + CTILE + e * CT + threadIdx.x, ic = i < on ? i : on - 1;
                okey[e] = __builtin_nontemporal_load(a.old_keys + ob + ic);
            }
        __syncthreads();
        const uint64_t last = tile[nt - 1];
        for (int q = threadIdx.x; q < u; q += CT) {
            const uint64_t key = nk[q];
            if (key <= last && (t0 == 0 || key > prev_last)) {
                const int L = lower_rank(tile, nt, key);
                a.w_lb[base + q] = (int)(t0 + L);
                fp[q] = 2 | (tile[L] == key ? 1 : 0);
            }
        }
        prev_last = last;
        __syncthreads();
    }
    RSTAMP(4);
    // F: exclusive prefix of the found flags (thread t: the run [t c, t c + c))
    const int c = (u + CT - 1) / CT;
    const int r0 = min(u, (int)threadIdx.x * c), r1 = min(u, r0 + c);
    int run = 0;
    for (int i = r0; i < r1; ++i) run += fp[i] & 1;
    int tot;
    int acc = block_scan<CT, int>(run, wsum, tot);
    for (int i = r0; i < r1; ++i) {
        const int f = fp[i];
        a.w_keys[base + i] = nk[i];
        a.w_fp[base + i] = acc;
        if (!(f & 2)) a.w_lb[base + i] = (int)on;            // above every old key
        acc += f & 1;
    }
    if (threadIdx.x == 0) { a.w_ulen[j] = u; a.w_found[j] = tot; }
    RSTAMP(5);
}

// merged lengths -> offsets (one work-group; n_halos is a catalogue size)
__global__ __launch_bounds__(1024) void k_collate_offsets(const oa_collate_args a) {
    __shared__ int64_t wsum[17];
    int64_t carry = 0;
    for (int j0 = 0; j0 < a.n_halos; j0 += 1024) {
        const int j = j0 + threadIdx.x;
        int64_t v = 0;
        if (j < a.n_halos) v = (a.old_off[j + 1] - a.old_off[j]) + a.w_ulen[j] - a.w_found[j];
        int64_t tot;
        const int64_t ex = block_scan<1024, int64_t>(v, wsum, tot);
        if (j < a.n_halos) a.new_off[j] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) a.new_off[a.n_halos] = carry;
}

// one work-group per halo: the new keys, their F and counts in LDS (a.lds_keys slots);
// the old list streams through once, MU elements per thread per trip, every load of a
// trip issued before any store (the stores may alias the old list for the compiler,
// which would otherwise hold each trip's loads behind the previous trip's stores)
__global__ __launch_bounds__(CT) void k_collate_place(const oa_collate_args a) {
    extern __shared__ __attribute__((aligned(16))) char cl_smem[];
    uint64_t *nk = reinterpret_cast<uint64_t *>(cl_smem);   // [lds_keys]
    int *fp = reinterpret_cast<int *>(nk + a.lds_keys);      // [lds_keys + 1]
    int *nc = fp + a.lds_keys + 1;                           // [lds_keys]
    const int j = blockIdx.x;
    const int u = a.w_ulen[j];
    const int64_t base = a.new_base[j];
    const int64_t ob = a.old_off[j], on = a.old_off[j + 1] - ob;
    const int64_t no = a.new_off[j], ne = a.new_off[j + 1];
    // every store below goes to [no, ne) of the merged state (and the workspace rows read
    // to [base, base + u) of [0, n_new_cap)): a position outside it -- an inconsistent
    // workspace -- raises OA_POST_BOUNDS and is dropped
    if (u < 0 || u > a.lds_keys || (u > 0 && (base < 0 || base + u > a.n_new_cap)) ||
        ne - no < on || ne > a.n_old + a.n_new_cap) {
        if (threadIdx.x == 0 && a.status) atomicOr(a.status, (int32_t)OA_POST_BOUNDS);
        return;
    }
    bool oob = false;
    for (int q0 = 0; q0 < u; q0 += CL_U * CT) {
        uint64_t k[CL_U];
        int f[CL_U], c[CL_U];
#pragma unroll
        for (int e = 0; e < CL_U; ++e) {
            const int q = q0 + e * CT + (int)threadIdx.x, qc = q < u ? q : u - 1;
            k[e] = a.w_keys[base + qc];
            f[e] = a.w_fp[base + qc];
            c[e] = a.w_cnt[base + qc];
        }
#pragma unroll
        for (int e = 0; e < CL_U; ++e) {
            const int q = q0 + e * CT + (int)threadIdx.x;
            if (q < u) { nk[q] = k[e]; fp[q] = f[e]; nc[q] = c[e]; }
        }
    }
    if (threadIdx.x == 0) fp[u] = a.w_found[j];
    __syncthreads();
    constexpr int MU = OA_PLACE_MU;
    for (int64_t i0 = threadIdx.x; i0 < on; i0 += (int64_t)CT * MU) {
        uint64_t key[MU];
        int64_t cnt[MU];
#pragma unroll
        for (int e = 0; e < MU; ++e) {
            const int64_t i = i0 + (int64_t)e * CT, ic = i < on ? i : on - 1;
            key[e] = __builtin_nontemporal_load(a.old_keys + ob + ic);
            cnt[e] = __builtin_nontemporal_load(a.old_cnt + ob + ic);
        }
#pragma unroll
        for (int e = 0; e < MU; ++e) {
            const int64_t i = i0 + (int64_t)e * CT;
            if (i >= on) break;
            const int L = lower_rank(nk, u, key[e]);
            const bool eq = L < u && nk[L] == key[e];
            const int64_t pos = no + i + L - fp[L];
            if (pos < no || pos >= ne) { oob = true; continue; }
            // plain stores: the positions shift by one at every inserted key, so a wave's
            // stores straddle lines, which L2 merges (non-temporal: 1.6x the time)
            a.new_keys[pos] = key[e];
            a.new_cnt[pos] = cnt[e] + (eq ? (int64_t)nc[L] : 0);
        }
    }
    for (int q = threadIdx.x; q < u; q += CT) {
        if (fp[q + 1] != fp[q]) continue;                    // already in the old list
        const int64_t pos = no + a.w_lb[base + q] + (q - fp[q]);
        if (pos < no || pos >= ne) { oob = true; continue; }
        a.new_keys[pos] = nk[q];
        a.new_cnt[pos] = nc[q];
    }
    if (oob && a.status) atomicOr(a.status, (int32_t)OA_POST_BOUNDS);
}

template <int KIND>
void (*collate_rank_kernel(int lds_keys))(oa_collate_args) {
    static_assert(16 * CT >= CH, "k_collate_rank sorts at most 16 keys per thread");
    return lds_keys <= 2 * CT ? k_collate_rank<KIND, 2>
         : lds_keys <= 4 * CT ? k_collate_rank<KIND, 4>
         : lds_keys <= 8 * CT ? k_collate_rank<KIND, 8> : k_collate_rank<KIND, 16>;
}

__global__ __launch_bounds__(256) void k_keys_to_ids(const uint64_t *keys, int64_t n, int key_signed,
                                                     int out_kind, void *out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t v = key_signed ? keys[i] ^ SIGN : keys[i];
    if (out_kind == OA_ID_I64 || out_kind == OA_ID_U64) static_cast<uint64_t *>(out)[i] = v;
    else static_cast<uint32_t *>(out)[i] = (uint32_t)v;
}

// save_final_apsis_counts (:222-236): per element, its count in the final snapshot
__global__ __launch_bounds__(256) void k_retro_counts(const void *ids, int kind, int64_t n,
                                                      const int64_t *offs, const int64_t *hinds,
                                                      int n_seg, const void *ids_final,
                                                      const int64_t *final_off,
                                                      const int64_t *counts_final, double *out,
                                                      int32_t *status) {
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e >= n) return;
    double r = 0.0;
    if (n_seg > 0 && e >= offs[0] && e < offs[n_seg]) {
        const int sg = (kind == OA_ID_I64 || kind == OA_ID_I32) ? 1 : 0;
        const int h2 = seg_of(offs, n_seg, e);
        const int64_t h1 = hinds[h2];
        const uint64_t key = to_key(load_val(ids, e, kind), sg);
        int64_t L = final_off[h1], R = final_off[h1 + 1];
        const int64_t end = R;
        while (L < R) {
            const int64_t mid = (L + R) >> 1;
            if (to_key(load_val(ids_final, mid, kind), sg) < key) L = mid + 1; else R = mid;
        }
        if (L < end && to_key(load_val(ids_final, L, kind), sg) == key) r = (double)counts_final[L];
        else atomicOr(status, (int32_t)OA_POST_MISSING);
    }
    out[e] = r;
}

// ------------------------------------------------------------------ f4: central IDs
// radius key of particle p about the halo centre: dx in the promoted dtype TD,
// recenter_coordinates (utils.py:24-33) per dim in its comparison dtype, then
// region_coords (float64, progenitors.py:41) and sqrt(einsum) with the host's f64 tree
// (SQ = false: the bits of r^2 itself -- the same order, since sqrt is monotone, with
// ties of r possibly split; r_of() turns such a key into the radius key)
template <typename TX, typename TD, bool SQ = true>
__device__ __forceinline__ uint64_t radius_key(const TX (&x)[3], const double *c,
                                               const oa_central_args &a) {
    TD d[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) d[k] = (TD)x[k] - (TD)c[k];
    for (int k = 0; k < a.n_box_dims; ++k) {
        if (a.wrap_f64[k]) {
            double v = (double)d[k];
            if (v > a.half[k]) d[k] = (TD)(v - a.box[k]);
            v = (double)d[k];
            if (v < -a.half[k]) d[k] = (TD)(v + a.box[k]);
        } else {
            const TD h = (TD)a.half[k], b = (TD)a.box[k];
            if (d[k] > h) d[k] = d[k] - b;
            if (d[k] < -h) d[k] = d[k] + b;
        }
    }
    const double r0 = (double)d[0], r1 = (double)d[1], r2 = (double)d[2];
    const double p0 = r0 * r0, p1 = r1 * r1, p2 = r2 * r2;
    const double r = SQ ? sqrt((p0 + p2) + p1) : (p0 + p2) + p1;
    return (uint64_t)__double_as_longlong(r);   // r >= +0 or NaN: bit order = numeric order, NaN last
}
__device__ __forceinline__ uint64_t r_of(uint64_t k2) {
    return (uint64_t)__double_as_longlong(sqrt(__longlong_as_double((long long)k2)));
}

// Raw buffer loads (resource: 48-bit base, byte size; lanes past the size read 0), so a
// block's coordinates are addressed by one 32-bit lane offset plus a scalar offset per
// particle instead of a 64-bit address per load.
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x3 __attribute__((ext_vector_type(3)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
__device__ f32x3 pb_v3f32(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.v3f32");
__device__ f64x2 pb_v2f64(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.v2f64");
__device__ double pb_f64(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.f64");
__device__ __forceinline__ i32x4 post_rsrc(const void *p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((int32_t)((uint32_t)(a >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int32_t)bytes);
    r.w = 0x00020000;
    return r;
}
template <typename TX>
__device__ __forceinline__ void load_xyz(i32x4 r, uint32_t vo, uint32_t so, TX (&x)[3]) {
    if constexpr (sizeof(TX) == 4) {
        const f32x3 v = pb_v3f32(r, (int32_t)vo, (int32_t)so, 0);
        x[0] = v.x; x[1] = v.y; x[2] = v.z;
    } else {
        const f64x2 v = pb_v2f64(r, (int32_t)vo, (int32_t)so, 0);
        x[0] = v.x; x[1] = v.y; x[2] = pb_f64(r, (int32_t)(vo + 16u), (int32_t)so, 0);
    }
}

constexpr int KR = 12;                     // k_central: radius keys per thread in registers
constexpr int HB = 12;                     // k_central: digit bits of the threshold pass

// Rank of every candidate by (key, position) among the n of them (n <= 1024, keys
// broadcast from LDS): the sorted order without a sorting network's log^2 barriers.
// Every thread of the work-group at work: candidate c = t mod n
// counts the candidates of one of G = 1024 / n slices of [0, n) and adds its partial
// rank to acc[c] (LDS, zeroed here); then each candidate is placed.  Barriers inside.
__device__ __forceinline__ void rank_pairs_split(const uint64_t *s, const uint32_t *x, int n,
                                                 uint64_t *ds, uint32_t *dx, int *acc) {
    const int t = threadIdx.x;
    if (t < n) acc[t] = 0;
    __syncthreads();
    const int G = 1024 / n, L = (n + G - 1) / G;
    const int c = t % n, g = t / n;
    if (g < G) {
        const uint64_t k = s[c];
        const uint32_t i = x[c];
        const int j1 = min(n, (g + 1) * L);
        int r = 0, j = g * L;
        constexpr int RU = 8;
        for (; j + RU <= j1; j += RU) {
            uint64_t kj[RU];
            uint32_t xj[RU];
#pragma unroll
            for (int u = 0; u < RU; ++u) { kj[u] = s[j + u]; xj[u] = x[j + u]; }
#pragma unroll
            for (int u = 0; u < RU; ++u) r += (kj[u] < k || (kj[u] == k && xj[u] < i)) ? 1 : 0;
        }
        for (; j < j1; ++j) {
            const uint64_t kj = s[j];
            r += (kj < k || (kj == k && x[j] < i)) ? 1 : 0;
        }
        if (r) atomicAdd(&acc[c], r);
    }
    __syncthreads();
    if (t < n) {
        const int r = acc[t];
        ds[r] = s[t];
        dx[r] = x[t];
    }
}

// <= 64 VGPRs: two 1024-thread work-groups per CU, so one's barriers and sort overlap
// the other's loads
template <typename TX, typename TD>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8)))
void k_central(const oa_central_args a) {
    __shared__ uint64_t sk[SC];
    __shared__ uint32_t si[SC];
    __shared__ uint64_t rk[1024];              // candidates in rank order (n <= 1024)
    __shared__ uint32_t ri[1024];
    __shared__ int hist[1 << HB];
    __shared__ int wsum[17];
    __shared__ uint64_t s_prefix;
    __shared__ unsigned long long s_min, s_max;
    __shared__ int s_need, s_cnt, s_done, s_bin, s_cum;
    const int h = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int64_t off = a.offsets[h];
    const int m = (int)(a.offsets[h + 1] - off);
    const int k = m < a.n ? m : a.n;
    if (k <= 0) return;
    const TX *x = static_cast<const TX *>(a.coords);
    const double *c = a.positions + 3 * (int64_t)h;
    CSTAMP(0);
    if (tid == 0) { s_min = ~0ull; s_max = 0; s_cnt = 0; s_done = 0; }
    for (int d = tid; d < (1 << HB); d += 1024) hist[d] = 0;
    __syncthreads();
    bool fast = m <= KR * 1024;                // uniform
    uint64_t key[KR];
    if (fast) {
        // Fast path (blocks of <= KR * 1024): every radius key stays in its thread's
        // registers.  One histogram of the HB bits below the block's common key prefix
        // gives a threshold digit B whose keys, with every smaller one, hold the k
        // smallest; when those are <= SC they are sorted by (key, position) in LDS and
        // the first k taken -- the same k keys, in the same order, as the exact select
        // below, in one pass over the keys instead of up to eight.
        uint64_t lmin = ~0ull, lmax = 0;
        // every particle's loads in flight at once: one lane offset, a scalar offset per
        // particle (1024 particles apart), past-the-block lanes read 0 (key ~0 below)
        constexpr int LU = sizeof(TX) == 4 ? KR : 4;
        const i32x4 rx = post_rsrc(x + 3 * off, (uint32_t)m * 3u * (uint32_t)sizeof(TX));
        const uint32_t vo = (uint32_t)tid * 3u * (uint32_t)sizeof(TX);
#pragma unroll
        for (int u0 = 0; u0 < KR; u0 += LU) {
            TX xs[LU][3];
#pragma unroll
            for (int u = 0; u < LU; ++u)
                load_xyz<TX>(rx, vo, (uint32_t)(u0 + u) * 1024u * 3u * (uint32_t)sizeof(TX), xs[u]);
#pragma unroll
            for (int u = 0; u < LU; ++u) {
                const int i = (u0 + u) * 1024 + tid;
                key[u0 + u] = i < m ? radius_key<TX, TD, false>(xs[u], c, a) : ~0ull;
                if (i < m) {
                    lmin = key[u0 + u] < lmin ? key[u0 + u] : lmin;
                    lmax = key[u0 + u] > lmax ? key[u0 + u] : lmax;
                }
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t y = __shfl_xor(lmin, o), z = __shfl_xor(lmax, o);
            lmin = y < lmin ? y : lmin;
            lmax = z > lmax ? z : lmax;
        }
        CSTAMP(1);
        if (lane == 0 && tid < m) { atomicMin(&s_min, lmin); atomicMax(&s_max, lmax); }
        __syncthreads();
        CSTAMP(2);
        // The keys here are r^2 (no sqrt per particle): they select, and only the
        // selected get their radius, which orders them.
        if (k == m) {
#pragma unroll
            for (int u = 0; u < KR; ++u) {
                const int i = u * 1024 + tid;
                if (i < m) { sk[i] = r_of(key[u]); si[i] = (uint32_t)i; }
            }
        } else {
            const uint64_t diff = s_min ^ s_max;
            const int lo_fixed = diff ? 64 - __clzll((long long)diff) : 0;
            const int sh = lo_fixed > HB ? lo_fixed - HB : 0;
            const uint32_t mask = (1u << (lo_fixed - sh)) - 1u;
            // every key shares the bits above lo_fixed: its digit is (key >> sh) & mask
#pragma unroll
            for (int u = 0; u < KR; ++u)
                if (u * 1024 + tid < m) atomicAdd(&hist[(key[u] >> sh) & mask], 1);
            __syncthreads();
            CSTAMP(3);
            // the digit B where the running count reaches k (4 bins per thread)
            int h4[4], sum = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) { h4[q] = hist[4 * tid + q]; sum += h4[q]; }
            int tot;
            const int ex = block_scan<1024, int>(sum, wsum, tot);
            if (ex < k && ex + sum >= k) {
                int acc = ex, q = 0;
                for (; q < 3; ++q) {
                    if (acc + h4[q] >= k) break;
                    acc += h4[q];
                }
                s_bin = 4 * tid + q;
                s_cum = acc + h4[q];
                // The cut: every r^2 key <= the bin's top E, and past it to the end of the
                // run of keys whose sqrt equals sqrt(E) (a few more).  A key above the cut
                // then has a radius > sqrt(E) >= the k-th smallest radius (at least k keys
                // are <= E), so no particle left out can tie the k-th radius.
                const uint64_t pre = s_min & ~((1ull << lo_fixed) - 1ull);
                uint64_t e = pre | ((uint64_t)s_bin << sh) | ((1ull << sh) - 1ull);
                if (e < 0x7FF0000000000000ull) {          // finite r^2: extend the plateau
                    const uint64_t re = r_of(e);
                    for (int t = 0; t < 8 && e + 1 < 0x7FF0000000000000ull && r_of(e + 1) == re; ++t) ++e;
                }
                s_prefix = e;
            }
            __syncthreads();
            CSTAMP(4);
            const uint64_t cut = s_prefix;
            fast = s_cum <= SC;
            if (fast) {
#pragma unroll
                for (int u = 0; u < KR; ++u) {
                    const int i = u * 1024 + tid;
                    if (i < m && key[u] <= cut) {
                        const int p = atomicAdd(&s_cnt, 1);
                        if (p < SC) { sk[p] = r_of(key[u]); si[p] = (uint32_t)i; }
                    }
                }
                __syncthreads();
                fast = s_cnt <= SC;                       // the plateau added too many
            }
            if (!fast) {
                // too many keys at the threshold: the exact select over radius keys, from
                // global (its min / max: sqrt is monotone)
#pragma unroll
                for (int u = 0; u < KR; ++u) {
                    const int i = u * 1024 + tid;
                    if (i < m) a.scratch[off + i] = r_of(key[u]);
                }
                __syncthreads();
                if (tid == 0) { s_min = r_of(s_min); s_max = r_of(s_max); s_cnt = 0; }
            }
        }
        __syncthreads();
    } else {
        // larger blocks: keys through global scratch, four particles per thread per
        // trip (their coordinate loads all in flight before the first radius)
        uint64_t lmin = ~0ull, lmax = 0;
        constexpr int RU = 4;
        for (int i0 = tid; i0 < m; i0 += 1024 * RU) {
            TX xs[RU][3];
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                const int i = i0 + u * 1024;
                const int64_t p = off + (i < m ? i : 0);
#pragma unroll
                for (int d = 0; d < 3; ++d) xs[u][d] = x[3 * p + d];
            }
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                const int i = i0 + u * 1024;
                if (i >= m) break;
                const uint64_t kk = radius_key<TX, TD>(xs[u], c, a);
                lmin = kk < lmin ? kk : lmin;
                lmax = kk > lmax ? kk : lmax;
                a.scratch[off + i] = kk;
            }
        }
        if (tid < m) { atomicMin(&s_min, lmin); atomicMax(&s_max, lmax); }
        __syncthreads();
    }
    const int n_sorted = (fast && k < m) ? s_cnt : k;
    if (!fast) {
#define KEY(i) a.scratch[off + (i)]
        if (k == m) {
            for (int i = tid; i < m; i += 1024) { sk[i] = KEY(i); si[i] = i; }
        } else {
            // MSB-first radix select of the k-th smallest key.  Bits above the highest
            // bit where the block's min and max keys differ are common and skipped; each
            // pass histograms the next <= 8 bits of the keys still matching the fixed
            // prefix.  A pass whose chosen bin is taken whole ends the select early
            // (inclusive bound hi); otherwise T = the exact k-th key and `need` ties to
            // it are taken by position.
            const uint64_t diff = s_min ^ s_max;
            int lo_fixed = diff ? 64 - __clzll((long long)diff) : 0;    // bits below are free
            uint64_t prefix = lo_fixed >= 64 ? 0ull : (s_min & ~((1ull << lo_fixed) - 1ull));
            int need = k;
            while (lo_fixed > 0) {
                const int s = lo_fixed > 8 ? lo_fixed - 8 : 0;
                const int w = lo_fixed - s;
                for (int d = tid; d < 256; d += 1024) hist[d] = 0;
                __syncthreads();
                for (int i = tid; i < m; i += 1024) {
                    const uint64_t kk = KEY(i);
                    if (lo_fixed >= 64 || (kk >> lo_fixed) == (prefix >> lo_fixed))
                        atomicAdd(&hist[(kk >> s) & ((1u << w) - 1u)], 1);
                }
                __syncthreads();
                if (tid < 64) {
                    // wave 0 finds the bin holding the need-th key: 4 bins per lane, a
                    // wave prefix sum, the first lane whose running count reaches `need`
                    const int l = tid;
                    const int h0 = hist[4 * l], h1 = hist[4 * l + 1], h2 = hist[4 * l + 2],
                              h3 = hist[4 * l + 3];
                    const int sum = h0 + h1 + h2 + h3;
                    int incl = sum;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const int y = __shfl_up(incl, o);
                        if (l >= o) incl += y;
                    }
                    const uint64_t hitm = __ballot(incl >= need);
                    if (l == __ffsll((unsigned long long)hitm) - 1) {
                        int acc = incl - sum, q = 0;
                        const int hs[4] = {h0, h1, h2, h3};
                        for (; q < 3; ++q) {
                            if (acc + hs[q] >= need) break;
                            acc += hs[q];
                        }
                        s_prefix = prefix | ((uint64_t)(4 * l + q) << s);
                        s_need = need - acc;
                        s_done = hs[q] == need - acc;          // the whole bin is selected
                    }
                }
                __syncthreads();
                prefix = s_prefix;
                need = s_need;
                lo_fixed = s;
                if (s_done) break;
            }
            if (lo_fixed > 0) {                  // early end: every key <= hi, exactly k of them
                const uint64_t hi = prefix | ((1ull << lo_fixed) - 1ull);
                for (int i = tid; i < m; i += 1024) {
                    const uint64_t kk = KEY(i);
                    if (kk <= hi) {
                        const int p = atomicAdd(&s_cnt, 1);
                        sk[p] = kk;
                        si[p] = (uint32_t)i;
                    }
                }
                need = 0;
            }
            const uint64_t T = prefix;
            if (need > 0) {
                for (int i = tid; i < m; i += 1024) {
                    const uint64_t kk = KEY(i);
                    if (kk < T) {
                        const int p = atomicAdd(&s_cnt, 1);
                        sk[p] = kk;
                        si[p] = (uint32_t)i;
                    }
                }
            }
            __syncthreads();
            const int lt = s_cnt;                      // = k - need
            int taken = 0;                             // ties to T: lowest positions first
            for (int i0 = 0; i0 < m && taken < need; i0 += 1024) {
                const int i = i0 + tid;
                const int f = (i < m && KEY(i) == T) ? 1 : 0;
                int tt;
                const int e = block_scan<1024, int>(f, wsum, tt);
                if (f && taken + e < need) { sk[lt + taken + e] = T; si[lt + taken + e] = (uint32_t)i; }
                taken += tt;
            }
        }
#undef KEY
    }
    __syncthreads();
    CSTAMP(5);
    const uint32_t *order = si;
    if (n_sorted <= 1024) {
        // the histogram is dead here: it holds the partial ranks
        rank_pairs_split(sk, si, n_sorted, rk, ri, hist);
        order = ri;
    } else {
        int P = 1;
        while (P < n_sorted) P <<= 1;
        for (int i = n_sorted + tid; i < P; i += 1024) { sk[i] = ~0ull; si[i] = 0xFFFFFFFFu; }
        __syncthreads();
        bitonic_pairs<1024>(sk, si, P);
    }
    __syncthreads();
    CSTAMP(6);
    const int64_t o = a.out_offsets[h];
    for (int r = tid; r < k; r += 1024) {
        const int64_t src = off + order[r];
        if (a.id_bytes == 8)
            static_cast<uint64_t *>(a.out_ids)[o + r] = static_cast<const uint64_t *>(a.ids)[src];
        else
            static_cast<uint32_t *>(a.out_ids)[o + r] = static_cast<const uint32_t *>(a.ids)[src];
    }
    CSTAMP(7);
}

// ------------------------------------------------------------------ f4: main progenitors
// The table is built over the SMALL side (the tracked central IDs, ~n per descendant)
// and the halo members are streamed past it once.  A slot is {key, first tracked index,
// smallest member position holding the key}, 16 B; the table stays L2 / MALL resident.
constexpr uint64_t EMPTY = SIGN;          // INT64_MIN marks a free slot (rejected as an ID)
struct MpSlot { uint64_t key; uint32_t first; uint32_t hpos; };

__global__ __launch_bounds__(256) void k_mp_fill(MpSlot *tab, uint64_t cap, uint32_t *neg1,
                                                 uint32_t *filt, uint64_t fwords) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < cap) { tab[i].key = EMPTY; tab[i].first = 0xFFFFFFFFu; tab[i].hpos = 0xFFFFFFFFu; }
    if (i < fwords) filt[i] = 0u;
    if (i == 0) *neg1 = 0xFFFFFFFFu;
}
// a blocked Bloom filter over the tracked IDs, L2-resident: two bits in one 32-bit
// word per ID (high hash bits, independent of the table slot's low bits), so a member
// costs one filter read and the false-positive rate at 16 filter bits per ID is ~1.4 %
// instead of ~6 % with one bit; most halo members are not tracked and skip the probe
__device__ __forceinline__ uint32_t filt_word(uint64_t h, uint64_t fbits) {
    return (uint32_t)((h >> 32) & ((fbits >> 5) - 1));
}
__device__ __forceinline__ uint32_t filt_mask(uint64_t h) {
    return (1u << ((h >> 54) & 31)) | (1u << ((h >> 59) & 31));
}

// tracked value -> smallest index holding it (np.unique(return_index=True), :82)
__global__ __launch_bounds__(256) void k_mp_insert(const void *src, int kind, int64_t n,
                                                   MpSlot *tab, uint64_t cap, int32_t *status,
                                                   uint32_t *filt, uint64_t fbits) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t v = load_val(src, i, kind);
    if (v == EMPTY) { atomicOr(status, (int32_t)OA_POST_SENTINEL); return; }
    const uint64_t h = mix64(v);
    atomicOr(&filt[filt_word(h, fbits)], filt_mask(h));
    uint64_t s = h & (cap - 1);
    for (uint64_t t = 0; t < cap; ++t) {
        uint64_t cur = tab[s].key;
        if (cur == EMPTY)
            cur = atomicCAS((unsigned long long *)&tab[s].key, (unsigned long long)EMPTY,
                            (unsigned long long)v);
        if (cur == EMPTY || cur == v) { atomicMin(&tab[s].first, (uint32_t)i); return; }
        s = (s + 1) & (cap - 1);
    }
}

__device__ __forceinline__ int64_t mp_find(const MpSlot *tab, uint64_t cap, uint64_t v) {
    uint64_t s = mix64(v) & (cap - 1);
    for (uint64_t t = 0; t < cap; ++t) {
        const uint64_t cur = tab[s].key;
        if (cur == v) return (int64_t)s;
        if (cur == EMPTY) return -1;
        s = (s + 1) & (cap - 1);
    }
    return -1;
}

// stream the halo members once: a member whose ID is tracked records its position (the
// in1d(tracked, halo_pids) / myin1d(halo_pids, ...) join, :95-99); the position of a
// member equal to -1 is kept apart for the de-duplicated tracked entries (:83).
// MP_U members per thread, a grid stride apart (coalesced): all their loads and filter
// reads are issued before any is used, so the random L2 filter reads overlap.  A member
// that passes the filter (tracked, or a ~1.4 % false positive) goes to the work-group's
// own queue segment (an LDS counter, no global atomics) instead of being looked up
// here: the table read behind the stream would stall whole waves for a few active
// lanes.  k_mp_resolve looks the segments up with every lane busy; a full segment
// falls back to the lookup in place.
#ifndef OA_MP_U
#define OA_MP_U 8
#endif
#ifndef OA_MP_SEG
#define OA_MP_SEG 128       // queue entries per probe work-group (of 256 * MP_U members)
#endif
constexpr int MP_U = OA_MP_U;
constexpr int MP_SEG = OA_MP_SEG;
// KIND: the member ID kind, a template argument so the loads are plain and unconditional
// (index clamped to the last member): a load under a lane test or a kind switch waits
// for its data before the next one issues.
template <int KIND>
__global__ __launch_bounds__(256) void k_mp_probe(const void *hp, int64_t n,
                                                  MpSlot *tab, uint64_t cap, uint32_t *neg1,
                                                  const uint32_t *filt, uint64_t fbits,
                                                  uint32_t *q, uint32_t *qcnt) {
    __shared__ uint32_t lcnt;
    if (threadIdx.x == 0) lcnt = 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t p0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    uint32_t *seg = q + (uint64_t)blockIdx.x * MP_SEG;
    uint64_t v[MP_U];
    uint32_t m[MP_U], w[MP_U];
#pragma unroll
    for (int u = 0; u < MP_U; ++u) {
        const int64_t p = p0 + u * stride;
        v[u] = load_val_nt<KIND>(hp, p < n ? p : n - 1);
    }
#pragma unroll
    for (int u = 0; u < MP_U; ++u) {
        const uint64_t h = mix64(v[u]);
        m[u] = filt_mask(h);
        w[u] = filt[filt_word(h, fbits)];
    }
#pragma unroll
    for (int u = 0; u < MP_U; ++u) {
        const int64_t p = p0 + u * stride;
        if (p < n && v[u] == ~0ull) atomicMin(neg1, (uint32_t)p);
        const bool cand = p < n && (w[u] & m[u]) == m[u];
        const uint64_t bal = __ballot(cand);
        if (bal == 0ull) continue;                  // wave-uniform
        const int lane = __lane_id();
        const int leader = __ffsll((unsigned long long)bal) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&lcnt, (uint32_t)__popcll(bal));
        base = __shfl(base, leader);
        if (!cand) continue;
        const uint32_t slot = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
        if (slot < (uint32_t)MP_SEG) { seg[slot] = (uint32_t)p; continue; }
        const int64_t s = mp_find(tab, cap, v[u]);
        if (s >= 0) atomicMin(&tab[s].hpos, (uint32_t)p);
    }
    __syncthreads();
    if (threadIdx.x == 0) qcnt[blockIdx.x] = lcnt < (uint32_t)MP_SEG ? lcnt : (uint32_t)MP_SEG;
}

// the queued candidates: table lookup, smallest member position per tracked key.  One
// thread per queue slot (a segment's unused slots exit at once): every lookup chain
// is in flight together, none waits behind another segment's
__global__ __launch_bounds__(256) void k_mp_resolve(const void *hp, int kind, MpSlot *tab,
                                                    uint64_t cap, const uint32_t *q,
                                                    const uint32_t *qcnt, uint32_t nseg) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t g = i / (uint64_t)MP_SEG;
    if (g >= nseg || (uint32_t)(i % (uint64_t)MP_SEG) >= qcnt[g]) return;
    const uint32_t p = q[i];
    const int64_t s = mp_find(tab, cap, load_val(hp, p, kind));
    if (s >= 0) atomicMin(&tab[s].hpos, p);
}

// per tracked entry: duplicates become -1 (:83-84), then the halo number of the member
// holding it (halo_number[inds], :92-102), or -1
__global__ __launch_bounds__(256) void k_mp_lookup(const oa_mainprog_args a, const MpSlot *tab,
                                                   uint64_t cap, const uint32_t *neg1, int32_t *hn) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= a.n_tracked) return;
    const uint64_t v = load_val(a.tracked, i, a.tracked_kind);
    const int64_t s = mp_find(tab, cap, v);
    uint32_t p = 0xFFFFFFFFu;
    if (s >= 0) p = tab[s].first == (uint32_t)i ? tab[s].hpos : *neg1;
    int32_t r = -1;
    if (p != 0xFFFFFFFFu && a.n_halos > 0 && a.halo_offsets[0] <= (int64_t)p)
        r = seg_of(a.halo_offsets, a.n_halos, (int64_t)p);
    hn[i] = r;
}

// per tracked block: plurality halo number, ties to the lowest (np.unique + argmax, :107-115)
__global__ __launch_bounds__(256) void k_mp_tally(const oa_mainprog_args a, const int32_t *hn,
                                                  int ts) {
    extern __shared__ uint32_t tab[];           // [ts] halo numbers, [ts] counts
    __shared__ unsigned long long best;
    uint32_t *tk = tab, *tc = tab + ts;
    const int b = blockIdx.x;
    for (int s = threadIdx.x; s < ts; s += 256) { tk[s] = 0xFFFFFFFFu; tc[s] = 0; }
    if (threadIdx.x == 0) best = 0;
    __syncthreads();
    const int64_t lo = a.tracked_offsets[b], hi = a.tracked_offsets[b + 1];
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
        const int32_t h = hn[i];
        if (h < 0) continue;
        uint32_t s = (uint32_t)(mix64((uint64_t)h) & (uint64_t)(ts - 1));
        int t = 0;
        for (; t < ts; ++t) {
            uint32_t cur = tk[s];
            if (cur == 0xFFFFFFFFu) cur = atomicCAS(&tk[s], 0xFFFFFFFFu, (uint32_t)h);
            if (cur == 0xFFFFFFFFu || cur == (uint32_t)h) { atomicAdd(&tc[s], 1u); break; }
            s = (s + 1) & (uint32_t)(ts - 1);
        }
        if (t == ts) atomicOr(a.status, (int32_t)OA_POST_OVERFLOW);
    }
    __syncthreads();
    unsigned long long mine = 0;
    for (int s = threadIdx.x; s < ts; s += 256)
        if (tc[s]) {
            const unsigned long long v = ((unsigned long long)tc[s] << 32) | (0xFFFFFFFFull - tk[s]);
            mine = v > mine ? v : mine;
        }
    if (mine) atomicMax(&best, mine);
    __syncthreads();
    if (threadIdx.x == 0)
        a.result[b] = best ? (int64_t)(0xFFFFFFFFull - (best & 0xFFFFFFFFull)) : -1;
}

uint64_t pow2_at_least(uint64_t v, uint64_t lo) {
    uint64_t c = lo;
    while (c < v) c <<= 1;
    return c;
}
// filter: >= 16 bits per tracked ID (~6 % false positives), 4 KiB .. 4 MiB
#ifndef OA_MP_FB
#define OA_MP_FB 16         // filter bits per tracked ID
#endif
// candidate queue: MP_SEG entries per probe work-group, and its per-segment counts
uint64_t mp_segments(uint64_t n_halo_pids) {
    return (n_halo_pids + 256 * MP_U - 1) / (256 * MP_U);
}
uint64_t mp_filter_bits(uint64_t n_tracked) {
    uint64_t b = pow2_at_least(OA_MP_FB * n_tracked, 1ull << 15);
    return b > (1ull << 25) ? (1ull << 25) : b;
}

}  // namespace

extern "C" {

// Diagnostic builds (-DOA_STAMPS=1 / 2): k_central's / k_collate_rank's per-block phase
// stamps of its last launch (8 per block, s_memrealtime at 100 MHz); returns the count
// copied or -1.
int64_t oa_debug_central_stamps(uint64_t *host, int64_t n) {
#if OA_STAMPS
    const int64_t m = n < (int64_t)CST_MAX * CST_N ? n : (int64_t)CST_MAX * CST_N;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cstamps), m * sizeof(uint64_t)) != hipSuccess) return -1;
    return m;
#else
    (void)host; (void)n;
    return -1;
#endif
}


int64_t oa_post_struct_size(int32_t which) {
    switch (which) {
        case 0: return sizeof(oa_collate_args);
        case 1: return sizeof(oa_central_args);
        case 2: return sizeof(oa_mainprog_args);
        default: return -1;
    }
}

int oa_collate_step(const oa_collate_args *args, void *stream) {
    oa_internal_error(nullptr);
    if (!args) return fail(OA_E_ARG, "oa_collate_step: null args");
    const oa_collate_args &a = *args;
    if (a.n_halos <= 0) return OA_OK;
    if (a.in_kind < 0 || a.in_kind > 3) return fail(OA_E_ARG, "oa_collate_step: bad id kind");
    if (!a.src_off || !a.src_cnt || !a.new_base || !a.old_off || !a.new_off || !a.w_ulen ||
        !a.w_found || (a.n_new_cap > 0 && (!a.apsis_ids || !a.angles || !a.keep_lut || !a.w_keys ||
                                            !a.w_cnt || !a.w_lb || !a.w_fp)) ||
        (a.n_old > 0 && (!a.old_keys || !a.old_cnt)) ||
        (a.n_old + a.n_new_cap > 0 && (!a.new_keys || !a.new_cnt)))
        return fail(OA_E_ARG, "oa_collate_step: null pointer");
    if (a.lds_keys < 64 || a.lds_keys > CH || (a.lds_keys & (a.lds_keys - 1)))
        return fail(OA_E_ARG, "oa_collate_step: lds_keys must be a power of two in [64, CHUNK]");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t lds1 = (int64_t)a.lds_keys * 8 +
                         (int64_t)(a.lds_keys + 1 > 2 * CTILE ? a.lds_keys + 1 : 2 * CTILE) * 4 +
                         ((int64_t)a.lds_keys + 1) * 4;
    const int64_t lds3 = (int64_t)a.lds_keys * 12 + ((int64_t)a.lds_keys + 1) * 4;
    auto krank = a.in_kind == OA_ID_I64 ? collate_rank_kernel<OA_ID_I64>(a.lds_keys)
               : a.in_kind == OA_ID_U64 ? collate_rank_kernel<OA_ID_U64>(a.lds_keys)
               : a.in_kind == OA_ID_I32 ? collate_rank_kernel<OA_ID_I32>(a.lds_keys)
                                        : collate_rank_kernel<OA_ID_U32>(a.lds_keys);
    if (hipFuncSetAttribute(reinterpret_cast<const void *>(krank),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void *>(k_collate_place),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds3) != hipSuccess)
        return fail(OA_E_LAUNCH, "oa_collate_step: hipFuncSetAttribute");
    if (a.phases < 0 || a.phases > 3) return fail(OA_E_ARG, "oa_collate_step: phases must be 0-3");
    const int ph = a.phases == 0 ? 3 : a.phases;
    if (ph & 1) {
        hipLaunchKernelGGL(krank, dim3(a.n_halos), dim3(CT), (size_t)lds1, st, a);
        if (int rc = check_launch("k_collate_rank")) return rc;
    }
    if (!(ph & 2)) return OA_OK;
    hipLaunchKernelGGL(k_collate_offsets, dim3(1), dim3(1024), 0, st, a);
    if (int rc = check_launch("k_collate_offsets")) return rc;
    if (a.n_old + a.n_new_cap > 0) {
        hipLaunchKernelGGL(k_collate_place, dim3(a.n_halos), dim3(CT), (size_t)lds3, st, a);
        if (int rc = check_launch("k_collate_place")) return rc;
    }
    return OA_OK;
}

int oa_keys_to_ids(const uint64_t *keys, int64_t n, int32_t key_signed, int32_t out_kind,
                   void *out, void *stream) {
    oa_internal_error(nullptr);
    if (n <= 0) return OA_OK;
    if (!keys || !out || out_kind < 0 || out_kind > 3) return fail(OA_E_ARG, "oa_keys_to_ids: bad args");
    hipLaunchKernelGGL(k_keys_to_ids, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), keys, n, key_signed, out_kind, out);
    return check_launch("k_keys_to_ids");
}

int oa_retro_counts(const void *ids, int32_t kind, int64_t n, const int64_t *offs,
                    const int64_t *hinds, int32_t n_seg, const void *ids_final,
                    const int64_t *final_off, const int64_t *counts_final,
                    double *out, int32_t *status, void *stream) {
    oa_internal_error(nullptr);
    if (n <= 0) return OA_OK;
    if (kind < 0 || kind > 3) return fail(OA_E_ARG, "oa_retro_counts: bad id kind");
    if (!ids || !out || !status || (n_seg > 0 && (!offs || !hinds || !final_off || !counts_final ||
                                                  !ids_final)))
        return fail(OA_E_ARG, "oa_retro_counts: null pointer");
    hipLaunchKernelGGL(k_retro_counts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), ids, kind, n, offs, hinds, n_seg,
                       ids_final, final_off, counts_final, out, status);
    return check_launch("k_retro_counts");
}

int oa_central_ids(const oa_central_args *args, void *stream) {
    oa_internal_error(nullptr);
    if (!args) return fail(OA_E_ARG, "oa_central_ids: null args");
    const oa_central_args &a = *args;
    if (a.n_halos <= 0 || a.n <= 0) return OA_OK;
    if (a.n > SC) return fail(OA_E_ARG, "oa_central_ids: n exceeds OA_CENTRAL_MAX_N");
    if (a.id_bytes != 4 && a.id_bytes != 8) return fail(OA_E_ARG, "oa_central_ids: id_bytes");
    if (a.n_box_dims < 0 || a.n_box_dims > 3) return fail(OA_E_ARG, "oa_central_ids: box dims");
    if (a.coord_f64 && !a.dx_f64) return fail(OA_E_ARG, "oa_central_ids: dx narrower than coordinates");
    if (!a.coords || !a.positions || !a.ids || !a.offsets || !a.out_offsets || !a.out_ids)
        return fail(OA_E_ARG, "oa_central_ids: null pointer");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (a.coord_f64)
        hipLaunchKernelGGL((k_central<double, double>), dim3(a.n_halos), dim3(1024), 0, st, a);
    else if (a.dx_f64)
        hipLaunchKernelGGL((k_central<float, double>), dim3(a.n_halos), dim3(1024), 0, st, a);
    else
        hipLaunchKernelGGL((k_central<float, float>), dim3(a.n_halos), dim3(1024), 0, st, a);
    return check_launch("k_central");
}

int64_t oa_mainprog_workspace_bytes(int64_t n_halo_pids, int64_t n_tracked) {
    // the halo members are streamed, not tabled: they size only the candidate queue
    const uint64_t nt = (uint64_t)(n_tracked > 0 ? n_tracked : 1);
    const uint64_t nh = (uint64_t)(n_halo_pids > 0 ? n_halo_pids : 0);
    const uint64_t ct = pow2_at_least(2 * nt, 64);
    return (int64_t)(ct * sizeof(MpSlot) + 64 + 4 * nt + 4 + mp_filter_bits(nt) / 8 +
                     4 * mp_segments(nh) * (MP_SEG + 1));
}

int oa_main_progenitors(const oa_mainprog_args *args, void *stream) {
    oa_internal_error(nullptr);
    if (!args) return fail(OA_E_ARG, "oa_main_progenitors: null args");
    const oa_mainprog_args &a = *args;
    if (a.n_blocks <= 0) return OA_OK;
    for (int k : {a.halo_kind, a.tracked_kind})
        if (k != OA_ID_I64 && k != OA_ID_I32 && k != OA_ID_U32)
            return fail(OA_E_ARG, "oa_main_progenitors: IDs must be int64, int32 or uint32");
    if (a.n_halo_pids >= 0xFFFFFFFFll || a.n_tracked >= 0xFFFFFFFFll)
        return fail(OA_E_ARG, "oa_main_progenitors: more than 2^32-1 IDs");
    if (!a.tab_keys || !a.result || !a.status || !a.tracked_offsets ||
        (a.n_tracked > 0 && !a.tracked) || (a.n_halo_pids > 0 && (!a.halo_pids || !a.halo_offsets)))
        return fail(OA_E_ARG, "oa_main_progenitors: null pointer");
    if (reinterpret_cast<uintptr_t>(a.tab_keys) & 15)
        return fail(OA_E_ARG, "oa_main_progenitors: workspace must be 16-byte aligned");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const uint64_t ct = pow2_at_least(2 * (uint64_t)(a.n_tracked > 0 ? a.n_tracked : 1), 64);
    const uint64_t nt = (uint64_t)(a.n_tracked > 0 ? a.n_tracked : 1);
    const uint64_t fbits = mp_filter_bits(nt), fwords = fbits / 32;
    MpSlot *tab = reinterpret_cast<MpSlot *>(a.tab_keys);
    uint32_t *neg1 = reinterpret_cast<uint32_t *>(tab + ct);
    int32_t *hn = reinterpret_cast<int32_t *>(neg1 + 16);
    uint32_t *filt = reinterpret_cast<uint32_t *>(hn + nt + 1);
    const uint64_t nfill = ct > fwords ? ct : fwords;
    hipLaunchKernelGGL(k_mp_fill, dim3((unsigned)((nfill + 255) / 256)), dim3(256), 0, st, tab, ct,
                       neg1, filt, fwords);
    if (int rc = check_launch("k_mp_fill")) return rc;
    if (a.n_tracked > 0) {
        hipLaunchKernelGGL(k_mp_insert, dim3((unsigned)((a.n_tracked + 255) / 256)), dim3(256), 0,
                           st, a.tracked, a.tracked_kind, a.n_tracked, tab, ct, a.status, filt, fbits);
        if (int rc = check_launch("k_mp_insert")) return rc;
        if (a.n_halo_pids > 0) {
            // the queue segments after the filter, then their counts
            const uint64_t nseg = mp_segments((uint64_t)a.n_halo_pids);
            uint32_t *q = filt + fwords, *qcnt = q + nseg * MP_SEG;
            auto probe = a.halo_kind == OA_ID_I64 ? k_mp_probe<OA_ID_I64>
                       : a.halo_kind == OA_ID_I32 ? k_mp_probe<OA_ID_I32> : k_mp_probe<OA_ID_U32>;
            hipLaunchKernelGGL(probe, dim3((unsigned)nseg), dim3(256), 0, st, a.halo_pids,
                               a.n_halo_pids, tab, ct, neg1, filt, fbits, q, qcnt);
            if (int rc = check_launch("k_mp_probe")) return rc;
            hipLaunchKernelGGL(k_mp_resolve, dim3((unsigned)((nseg * MP_SEG + 255) / 256)), dim3(256), 0,
                               st, a.halo_pids, a.halo_kind, tab, ct, q, qcnt, (uint32_t)nseg);
            if (int rc = check_launch("k_mp_resolve")) return rc;
        }
        hipLaunchKernelGGL(k_mp_lookup, dim3((unsigned)((a.n_tracked + 255) / 256)), dim3(256), 0,
                           st, a, tab, ct, neg1, hn);
        if (int rc = check_launch("k_mp_lookup")) return rc;
    }
    int ts = 64;
    while (ts < 2 * a.max_block && ts < 16384) ts <<= 1;
    if (hipFuncSetAttribute(reinterpret_cast<const void *>(k_mp_tally),
                            hipFuncAttributeMaxDynamicSharedMemorySize, ts * 8) != hipSuccess)
        return fail(OA_E_LAUNCH, "oa_main_progenitors: hipFuncSetAttribute");
    hipLaunchKernelGGL(k_mp_tally, dim3(a.n_blocks), dim3(256), (size_t)ts * 8, st, a, hn, ts);
    return check_launch("k_mp_tally");
}

}  // extern "C"
