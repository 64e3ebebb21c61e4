// Equihash solver for CDNA4 (gfx950) — the GPU replacement for the reference's
// CPU BasicSolve/OptimisedSolve (reference src/crypto/equihash.cpp:332-722,
// called from generateBlocks src/rpc/mining.cpp:161-199).
//
// Design: an atomic-free, bucket-sorted Wagner solver with parent pointers.
//
//  * Rows are bucketed on the top BB bits of the current digit (NB = 2^BB buckets,
//    ~INIT/NB rows each; (200,9): 512 buckets x 4096 rows).
//  * Every kernel launch is "one workgroup per bucket". A workgroup owns an output
//    AREA of CAP row slots. Instead of a global atomic per emitted row (memory-side
//    atomics across the 8 XCDs measured ~15 G/s, which dominated round time in the
//    first version), each workgroup counting-sorts its outputs by destination bucket
//    IN LDS and writes
//      - the rows into its own area, grouped by destination bucket,
//      - one column of the NB x NB count/offset matrices CNT[dest][src], OFF[dest][src].
//    The next round's workgroup `d` reads row d of those matrices and gathers its NB
//    contiguous runs (lane per row) straight into LDS. Outputs are permuted in LDS so
//    each workgroup writes its area in slot order (lane-consecutive, coalesced stores).
//  * Collisions on the remaining RB = DB-BB bits of the digit are found with an LDS
//    hash table (atomicExch chain heads); each row keeps a 64-bit parent reference
//    (global slot of both parents), so nothing ever carries index lists.
//  * Depth-1 duplicate pruning: pairs whose rows share a parent are dropped.
//  * Final round: pairs equal on all remaining bits are candidates; eh_expand walks
//    the K levels of parent references, canonicalises subtree order (reference
//    IsValidSolution ordering rule) and rejects repeated indices (LDS bitonic sort).
//
// Memory traffic per row per round: one coalesced gather, one area write, one 8-byte
// reference write. No global atomics except the (rare) candidate append.
#include <hip/hip_runtime.h>

#include "crypto/hashes.h"
#include "kernels/blake2b_device.h"
#include "kernels/gpu_api.h"
#include "kernels/hip_util.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <utility>

namespace bcpk {

template <int N_, int K_, int BB_, int CAP_, int NT_, int GENWG_, int NTG_, int MAXCAND_, int CAP4_ = CAP_,
          int CAP3_ = CAP_>
struct EhCfg {
    static constexpr int N = N_, K = K_;
    static constexpr int DB = N / (K + 1);           // digit bits
    static constexpr int BB = BB_;                   // bucket bits
    static constexpr int RB = DB - BB_;              // in-bucket collision bits
    static constexpr int NB = 1 << BB_;              // buckets (= output areas of rounds 1..K-1)
    static constexpr int NRESTS = 1 << RB;
    // LDS row capacity of a round by the width of the rows it reads: the narrow late rounds
    // hold more rows (their buckets and pair lists overflow most, from duplicate subtrees)
    static constexpr int CAP = CAP_;                 // rounds reading >= 5-word rows
    static constexpr int cap(int round) {
        return words(round - 1) >= 5 ? CAP_ : words(round - 1) == 4 ? CAP4_ : CAP3_;
    }
    static constexpr int AREA = CAP_ > CAP4_ ? (CAP_ > CAP3_ ? CAP_ : CAP3_) : (CAP4_ > CAP3_ ? CAP4_ : CAP3_);
    static constexpr int NT = NT_;                   // threads per round workgroup
    static constexpr int NW = NT_ / 64;
    static constexpr int INIT = 1 << (DB + 1);
    static constexpr int GENWG = GENWG_;             // generation workgroups (= stage-0 areas)
    static constexpr int NTG = NTG_;                 // threads per generation workgroup
    static constexpr int RPW = INIT / GENWG_;        // rows per generation workgroup
    static constexpr int IPH = 512 / N;
    static constexpr int NBYTES = N / 8;
    static constexpr int MAXCAND = MAXCAND_;
    static constexpr int L = 1 << K;
    static constexpr int bits(int stage) { return N - stage * DB - BB_; }
    static constexpr int words(int stage) { return (bits(stage) + 31) / 32; }
    static constexpr int WMAX = words(0);
    static constexpr int nsrc(int stage) { return stage == 0 ? GENWG_ : NB; } // areas holding stage rows
    static constexpr size_t ROWS = (size_t)NB * AREA; // slots per stage per nonce (>= GENWG*RPW)
    static_assert((size_t)GENWG_ * RPW <= ROWS && RPW * GENWG_ == INIT, "generation areas");
    static_assert(RB > 0 && DB < 32, "digit geometry");
    static_assert(AREA < 8192 && RPW < 65535, "u16 indices, 13-bit parent signatures");
    static_assert(NT_ % 64 == 0 && 4 * NT_ >= GENWG_ && 4 * NT_ >= NB && 4 * NTG_ >= NB, "workgroup shape");
    static_assert(words(K - 1) == 1, "final round keeps whole rows in one LDS word");
};

// Mainnet/testnet (200,9); (96,5); regtest (48,5).
using Cfg200_9 = EhCfg<200, 9, 9, 4416, 1024, 512, 1024, 256, 4864, 5120>;
using Cfg96_5 = EhCfg<96, 5, 7, 1280, 256, 256, 256, 256>;
using Cfg48_5 = EhCfg<48, 5, 3, 256, 64, 8, 64, 256>;

constexpr uint32_t NIL16 = 0xffffu;
constexpr uint32_t NIL = 0xffffffffu;
constexpr int MAX_CHAIN = 48;

// Block-wide scans over n (<= MAXPER*NT) values in LDS `v`, in place; each thread owns `per`
// consecutive entries, waves scan with shuffles, wave totals are combined through `wsum`
// (>= NT/64 + 1 entries).
// Exclusive sum (entries of type T: u32, or u16 when every prefix fits). Returns the total.
template <int NT, int MAXPER = 4, class T = uint32_t>
__device__ uint32_t block_exscan(T* v, int n, uint32_t* wsum) {
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int per = (n + NT - 1) / NT;
    uint32_t local[MAXPER];
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < MAXPER; ++q) {
        const int i = tid * per + q;
        local[q] = (q < per && i < n) ? (uint32_t)v[i] : 0u;
        s += local[q];
    }
    uint32_t x = s; // wave inclusive scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < NW; ++w) {
            const uint32_t t = wsum[w];
            wsum[w] = acc;
            acc += t;
        }
        wsum[NW] = acc;
    }
    __syncthreads();
    uint32_t base = wsum[wid] + x - s;
#pragma unroll
    for (int q = 0; q < MAXPER; ++q) {
        const int i = tid * per + q;
        if (q < per && i < n) v[i] = (T)base;
        base += local[q];
    }
    const uint32_t total = wsum[NW];
    __syncthreads();
    return total;
}

// Inclusive prefix maximum (entries u32 or u16).
template <int NT, int MAXPER = 4, class T = uint32_t>
__device__ void block_maxscan(T* v, int n, uint32_t* wsum) {
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int per = (n + NT - 1) / NT;
    uint32_t local[MAXPER];
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < MAXPER; ++q) {
        const int i = tid * per + q;
        local[q] = (q < per && i < n) ? (uint32_t)v[i] : 0u;
        s = max(s, local[q]);
    }
    uint32_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x = max(x, y);
    }
    const uint32_t excl = __shfl_up(x, 1, 64);
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < NW; ++w) {
            const uint32_t t = wsum[w];
            wsum[w] = acc;
            acc = max(acc, t);
        }
    }
    __syncthreads();
    uint32_t run = max(wsum[wid], lane ? excl : 0u);
#pragma unroll
    for (int q = 0; q < MAXPER; ++q) {
        const int i = tid * per + q;
        run = max(run, local[q]);
        if (q < per && i < n) v[i] = (T)run;
    }
    __syncthreads();
}

// ------------------------------------------------------------------ stage 0
// Generation workgroup gw hashes rows [gw*RPW, (gw+1)*RPW), counting-sorts them by bucket in
// LDS and writes its area in slot order (lane-consecutive stores) + column gw of CNT/OFF
// (CNT0/OFF0 are NB x GENWG).
template <class C, bool HDR>
__global__ __launch_bounds__(C::NTG) void eh_gen(const EhBaseState* __restrict__ states, uint32_t* __restrict__ R,
                                                 uint32_t* __restrict__ F, uint32_t* __restrict__ CNT,
                                                 uint32_t* __restrict__ OFF) {
    constexpr int W0 = C::words(0);
    constexpr int SW = (C::N + 31) / 32 + 1;
    constexpr int NTG = C::NTG;
    __shared__ uint32_t rows[C::RPW * W0];
    __shared__ uint16_t dst[C::RPW];
    __shared__ uint16_t perm[C::RPW];
    __shared__ uint32_t hist[C::NB], cur[C::NB];
    __shared__ uint32_t wsum[NTG / 64 + 1];
    const int gw = blockIdx.x % C::GENWG;
    const int nonce = blockIdx.x / C::GENWG;
    const int tid = threadIdx.x;
    const EhBaseState& bs = states[nonce];
    for (int i = tid; i < C::NB; i += NTG) hist[i] = 0;
    __syncthreads();
    const uint32_t r0 = (uint32_t)gw * C::RPW, r1 = r0 + C::RPW;
    const uint32_t g0 = r0 / C::IPH, g1 = (r1 + C::IPH - 1) / C::IPH;
    for (uint32_t g = g0 + tid; g < g1; g += NTG) {
        uint64_t h[8];
        if constexpr (HDR) eh_hash_g_hdr(bs, g, h);
        else eh_hash_g(bs, g, h);
#pragma unroll
        for (int s = 0; s < C::IPH; ++s) {
            const uint32_t idx = g * C::IPH + s;
            if (idx < r0 || idx >= r1) continue;
            uint32_t S[SW];
#pragma unroll
            for (int w = 0; w < SW; ++w) {
                uint32_t v = 0;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int k = 4 * w + t;
                    v = (v << 8) | ((k < C::NBYTES) ? digest_byte(h, s * C::NBYTES + k) : 0u);
                }
                S[w] = v;
            }
            const uint32_t li = idx - r0;
            const uint32_t d = S[0] >> (32 - C::BB);
#pragma unroll
            for (int w = 0; w < W0; ++w) rows[li * W0 + w] = (S[w] << C::BB) | (S[w + 1] >> (32 - C::BB));
            dst[li] = (uint16_t)d;
            atomicAdd(&hist[d], 1u);
        }
    }
    __syncthreads();
    for (int i = tid; i < C::NB; i += NTG) cur[i] = hist[i];
    __syncthreads();
    block_exscan<NTG>(cur, C::NB, wsum); // cur = run offsets inside area gw
    uint32_t* cntp = CNT + (size_t)nonce * C::NB * C::GENWG;
    uint32_t* offp = OFF + (size_t)nonce * C::NB * C::GENWG;
    for (int i = tid; i < C::NB; i += NTG) {
        cntp[(size_t)i * C::GENWG + gw] = hist[i];
        offp[(size_t)i * C::GENWG + gw] = cur[i];
    }
    __syncthreads();
    for (int li = tid; li < C::RPW; li += NTG) perm[atomicAdd(&cur[dst[li]], 1u)] = (uint16_t)li;
    __syncthreads();
    // word-flat stores: consecutive lanes write consecutive dwords of the area
    uint32_t* area = R + ((size_t)nonce * C::ROWS + (size_t)gw * C::RPW) * C::WMAX;
    uint32_t* farea = F + (size_t)nonce * C::ROWS + (size_t)gw * C::RPW;
    for (int k = tid; k < C::RPW * W0; k += NTG) {
        const uint32_t t = k / W0, w = k - t * W0;
        area[k] = rows[perm[t] * W0 + w];
    }
    for (int t = tid; t < C::RPW; t += NTG) farea[t] = r0 + perm[t];
}

// ------------------------------------------------------------------ stages 1..K
__device__ __forceinline__ bool share_parent(uint64_t a, uint64_t b) {
    const uint32_t a0 = (uint32_t)(a >> 32), a1 = (uint32_t)a, b0 = (uint32_t)(b >> 32), b1 = (uint32_t)b;
    return a0 == b0 || a0 == b1 || a1 == b0 || a1 == b1;
}

// index of the run holding LDS row r: last b with start[b] <= r (start is non-decreasing)
template <int NS> __device__ __forceinline__ uint32_t run_of(const uint32_t* start, uint32_t r) {
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = NS / 2; step > 0; step >>= 1)
        if (start[lo + step] <= r) lo += step;
    return lo;
}

// Diagnostic builds (STAMP) record s_memtime at each phase boundary (thread 0, after the
// barrier) into `stamps` — never used by the production instantiation.
#define EH_STAMP(k)                                                                                  \
    do {                                                                                             \
        if constexpr (STAMP) {                                                                       \
            if (threadIdx.x == 0) stamps[(size_t)bk * 16 + (k)] = __builtin_amdgcn_s_memtime();        \
        }                                                                                            \
    } while (0)

// LDS bytes of a persistent round (one 1024-lane workgroup per CU for (200,9)).
// Phase-D union (bytes): walk {sidx[CAP] u16, bend[NRESTS] u32, offp[CAP] u16};
// prefetch {gslot[CAP] u32}.
template <class C> constexpr int un_walk_bend(int cap) { return (cap * 2 + 3) / 4 * 4; }
template <class C> constexpr int un_walk_offp(int cap) { return un_walk_bend<C>(cap) + C::NRESTS * 4; }
template <class C> constexpr int round_un(int cap) {
    const int walk = un_walk_offp<C>(cap) + cap * 2;
    const int pref = cap * 4;
    return walk > pref ? walk : pref;
}
template <class C> constexpr int round_lds(int stage, bool prune) {
    const int WI = C::words(stage - 1);
    const int NS = C::nsrc(stage - 1);
    const int cap = C::cap(stage);
    const int marks = stage == C::K ? 0 : (C::AREA + C::NT - 1) / C::NT * C::NT * 2;
    return cap * WI * 4 + (prune ? cap * 4 : 0) + marks + round_un<C>(cap) +
           2 * (2 * NS + 1) * 4 + 2 * C::NB * 4 + 256;
}
// Depth-1 duplicate pruning wherever its signatures fit next to the full rows.
template <class C> constexpr bool round_prunes(int stage) {
    return stage >= 2 && round_lds<C>(stage, true) <= 160 * 1024;
}

// Parent references. A stage-s row (s >= 1) at global slot g = d*AREA + t stores
// F = (j << 16) | i: it was made in round s by workgroup d (= g / AREA, implied by the slot)
// from its LDS rows i and j. Round s also records its gather map M_s[d*AREA + r] = global
// slot (stage s-1) of LDS row r, so the index tree is walked as
// slot -> (d, F) -> (d,i,j) -> M -> parent slots. Stage-0 F holds leaf indices.
__device__ __forceinline__ uint64_t pack_tri(uint32_t d, uint32_t i, uint32_t j) {
    return ((uint64_t)d << 32) | (j << 16) | i;
}
// 2 x 16-bit signature of a row's parents for depth-1 duplicate pruning: each half is the
// parent's LDS row (13 bits) plus 3 bits of the producing workgroup. A half shared by two rows
// is confirmed exactly by comparing the full producing workgroups (from the run table): a
// signature-only prune would drop ~1e-4 of all pairs, ~6% of the solutions (511 pairs each).
__device__ __forceinline__ uint32_t parent_sig(uint32_t d, uint32_t f) {
    const uint32_t i = f & 0x1fff, j = (f >> 16) & 0x1fff;
    return ((i | ((d & 7) << 13)) << 16) | (j | ((d & 7) << 13));
}

// Row I/O of W dwords at a dword-aligned byte offset through a buffer descriptor: one
// 16-byte access plus a remainder (dword-aligned 16-byte buffer accesses are legal on gfx950).
template <int W> __device__ __forceinline__ void row_load(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t* o) {
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u3 __attribute__((ext_vector_type(3)));
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    if constexpr (W >= 4) {
        const u4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
        o[0] = x.x, o[1] = x.y, o[2] = x.z, o[3] = x.w;
        row_load<W - 4>(rs, off + 16, o + 4);
    } else if constexpr (W == 3) {
        const u3 x = __builtin_amdgcn_raw_buffer_load_b96(rs, off, 0, 0);
        o[0] = x.x, o[1] = x.y, o[2] = x.z;
    } else if constexpr (W == 2) {
        const u2 x = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
        o[0] = x.x, o[1] = x.y;
    } else if constexpr (W == 1) {
        o[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
    }
}
template <int W> __device__ __forceinline__ void row_store(__amdgpu_buffer_rsrc_t rs, uint32_t off, const uint32_t* v) {
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u3 __attribute__((ext_vector_type(3)));
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    if constexpr (W >= 4) {
        const u4 x = {v[0], v[1], v[2], v[3]};
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, off, 0, 0);
        row_store<W - 4>(rs, off + 16, v + 4);
    } else if constexpr (W == 3) {
        const u3 x = {v[0], v[1], v[2]};
        __builtin_amdgcn_raw_buffer_store_b96(x, rs, off, 0, 0);
    } else if constexpr (W == 2) {
        const u2 x = {v[0], v[1]};
        __builtin_amdgcn_raw_buffer_store_b64(x, rs, off, 0, 0);
    } else if constexpr (W == 1) {
        __builtin_amdgcn_raw_buffer_store_b32(v[0], rs, off, 0, 0);
    }
}

// STAGE < K: collision round producing stage-STAGE rows. STAGE == K: final round.
// Bucket bk = nonce*NB + d holds the stage STAGE-1 rows whose top digit bits are d; it becomes
// output area d of stage STAGE.
//
// The kernel is PERSISTENT and software-pipelined: one workgroup per CU walks buckets
// blockIdx.x, +gridDim.x, ... While it collides bucket b out of LDS, the rows of its next
// bucket are already in flight into VGPRs (plain loads are not drained by a bare barrier),
// and the run table of the bucket after that is in flight too. Per bucket:
//   A. commit: prefetched rows (VGPRs) -> LDS rows (+ parent signatures when pruning);
//   B. run table of the NEXT bucket from its prefetched CNT/OFF column (exclusive scan);
//      fetch the run table of the bucket after it (registers, not waited for);
//   C. slot map of the next bucket (16 lanes per run) -> gather map M; issue its row loads,
//      one lane per row, 16-byte buffer loads (not waited for);
//   D. collide bucket b: counting sort of the rows by their RB bits, atomic-free pair
//      enumeration (scan + max-scan, one lane per pair; depth-1 pruning), counting sort of the
//      pairs by destination, one-lane-per-row emit (XOR, shift one digit, 16-byte stores) in
//      slot order + one column of CNT/OFF.
template <class C, int STAGE, bool STAMP>
__global__ __launch_bounds__(C::NT) void eh_round(const uint32_t* __restrict__ Rin, const uint32_t* __restrict__ Fin,
                                                  const uint32_t* __restrict__ CNTin,
                                                  const uint32_t* __restrict__ OFFin, uint32_t* __restrict__ Rout,
                                                  uint32_t* __restrict__ Fout, uint32_t* __restrict__ CNTout,
                                                  uint32_t* __restrict__ OFFout, uint32_t* __restrict__ Mout,
                                                  uint32_t* __restrict__ ncand, uint64_t* __restrict__ cand,
                                                  uint64_t* __restrict__ stamps, uint32_t* __restrict__ pdrop,
                                                  int nbk) {
    constexpr int WI = C::words(STAGE - 1);
    constexpr int WO = (STAGE < C::K) ? C::words(STAGE) : 1;
    constexpr int NS = C::nsrc(STAGE - 1);
    constexpr int CAP = C::cap(STAGE);                        // LDS rows / pair-list entries
    constexpr int SSTRIDE = (STAGE == 1) ? C::RPW : C::AREA; // slots per source area
    constexpr bool FINAL = STAGE == C::K;
    constexpr bool PRUNE = round_prunes<C>(STAGE);
    static_assert(round_lds<C>(STAGE, PRUNE) <= 160 * 1024, "round LDS budget");
    constexpr int NT = C::NT;
    static_assert(NS <= NT, "one run-table entry per lane");
    constexpr int RPL = (CAP + NT - 1) / NT; // prefetched rows per lane
    // `un` is the phase-D union described at round_un().
    __shared__ uint32_t rows[CAP * WI];
    __shared__ uint32_t psig[PRUNE ? CAP : 1];
    constexpr int MP = FINAL ? 1 : (C::AREA + NT - 1) / NT; // pairs per lane (registers)
    constexpr int MPR = (CAP + NT - 1) / NT;                  // LDS rows per lane (scans)
    __shared__ uint16_t pmark[FINAL ? 1 : MP * NT];           // pair index -> first sorted position
    __shared__ __attribute__((aligned(16))) uint8_t un[round_un<C>(CAP)];
    __shared__ uint32_t rpos[2][NS + 1], rsrc[2][NS], hist[C::NB], cur[C::NB];
    __shared__ uint32_t wsum[C::NW + 1];
    uint32_t* gslot = reinterpret_cast<uint32_t*>(un);
    uint16_t* sidx = reinterpret_cast<uint16_t*>(un);
    uint32_t* bend = reinterpret_cast<uint32_t*>(un + un_walk_bend<C>(CAP));
    uint16_t* offp = reinterpret_cast<uint16_t*>(un + un_walk_offp<C>(CAP));
    const int tid = threadIdx.x;
    const int G = gridDim.x;
    int bk = blockIdx.x;
    if (bk >= nbk) return; // uniform per workgroup

    uint32_t rt_cnt = 0, rt_off = 0; // run-table entry `tid` of a bucket two steps ahead
    auto rt_fetch = [&](int bb) {
        if (bb < nbk && tid < NS) {
            const size_t at = (size_t)(bb / C::NB) * C::NB * NS + (size_t)(bb % C::NB) * NS + tid;
            rt_cnt = CNTin[at];
            rt_off = OFFin[at];
        }
    };
    auto rt_commit = [&](int p) -> uint32_t {
        if (tid < NS) {
            rpos[p][tid] = rt_cnt;
            rsrc[p][tid] = rt_off;
        }
        __syncthreads();
        const uint32_t total = block_exscan<NT>(rpos[p], NS, wsum);
        if (tid == 0) rpos[p][NS] = total;
        __syncthreads();
        return min(total, (uint32_t)CAP);
    };
    // A thread id the compiler cannot see through: keeps the per-lane index math of the
    // prefetch/commit loops from being hoisted out of the persistent loop (live invariants
    // would otherwise push the prefetched rows out to scratch).
    auto opaque_tid = [&]() -> uint32_t {
        uint32_t t;
        asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(tid));
        return t;
    };
    uint32_t v[RPL][WI];
    uint32_t f[PRUNE ? RPL : 1], fd[PRUNE ? RPL : 1]; // parent refs + producing workgroup
    uint32_t so[RPL];                                  // slots of the next bucket's rows
    int pf_nonce = 0, pf_d = 0;
    uint32_t pf_n = 0;
    auto prefetch = [&](int bb, int p, uint32_t nn) {
        const int nonce = bb / C::NB, d = bb % C::NB;
        { // slot of every LDS row: 16 lanes per run, 4 runs per wave instruction
            const int lane = tid & 63, wid = tid >> 6, sub = lane >> 4, l16 = lane & 15;
            for (int b0 = wid * 4; b0 < NS; b0 += C::NW * 4) {
                const int b = b0 + sub;
                if (b < NS) {
                    const uint32_t p0 = rpos[p][b];
                    const uint32_t len = rpos[p][b + 1] - p0;
                    const uint32_t s0 = b * SSTRIDE + rsrc[p][b];
                    for (uint32_t j = l16; j < len && p0 + j < nn; j += 16) gslot[p0 + j] = s0 + j;
                }
            }
        }
        __syncthreads();
        EH_STAMP(8);
        // buffer loads: 32-bit lane offsets against a per-nonce descriptor keep the address
        // math out of the VGPRs that hold the prefetched rows across phase D
        const auto rsrc_rows = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t*>(Rin + (size_t)nonce * C::ROWS * C::WMAX), 0, C::ROWS * C::WMAX * 4, 0x00020000);
        const auto rsrc_refs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(Fin + (size_t)nonce * C::ROWS),
                                                                 0, C::ROWS * 4, 0x00020000);
        const uint32_t ot = opaque_tid();
#pragma unroll
        for (int u = 0; u < RPL; ++u) {
            const uint32_t r = ot + u * NT;
            so[u] = (r < nn) ? gslot[r] : 0u; // clamped to a valid slot: loads are unconditional
        }
        pf_nonce = nonce;
        pf_d = d;
        pf_n = nn;
    };
    // Gather map of the prefetched bucket, from the slots held in registers: written late in
    // phase D, where its stores do not compete with the prefetch loads for the CU's queue.
    auto write_map = [&]() {
        uint32_t* mrow = Mout + (size_t)pf_nonce * C::ROWS + (size_t)pf_d * C::AREA;
        const uint32_t ot = opaque_tid();
#pragma unroll
        for (int u = 0; u < RPL; ++u) {
            const uint32_t r = ot + u * NT;
            if (r < pf_n) mrow[r] = so[u];
        }
    };
    // Issue the prefetch loads of rows [U0, U1) of every lane. The loads of one bucket are
    // issued in slices spread over phase D: a wave that issues the whole bucket at once stalls
    // at issue once the CU's outstanding-request window is full, and the barrier after it
    // then holds every other wave too.
    auto issue = [&](int u0, int u1) {
        const auto rsrc_rows = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t*>(Rin + (size_t)pf_nonce * C::ROWS * C::WMAX), 0, C::ROWS * C::WMAX * 4, 0x00020000);
        const auto rsrc_refs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t*>(Fin + (size_t)pf_nonce * C::ROWS), 0, C::ROWS * 4, 0x00020000);
#pragma unroll
        for (int u = 0; u < RPL; ++u) {
            if (u < u0 || u >= u1) continue;
            row_load<WI>(rsrc_rows, so[u] * (WI * 4), v[u]);
            if constexpr (PRUNE) {
                f[u] = __builtin_amdgcn_raw_buffer_load_b32(rsrc_refs, so[u] * 4, 0, 0);
                fd[u] = so[u] / C::AREA;
            }
        }
    };

    // prologue: run table of the first bucket, prefetch its rows, fetch the second run table
    int pb = 0;
    rt_fetch(bk);
    uint32_t n = rt_commit(0);
    rt_fetch(bk + G);
    prefetch(bk, 0, n);
    issue(0, RPL);
    write_map();
    __syncthreads();

    for (;;) {
        const int nonce = bk / C::NB, d = bk % C::NB;
        const size_t matout = (size_t)nonce * C::NB * C::NB;
        EH_STAMP(0);
        // A. commit the prefetched rows
        {
            const uint32_t ot = opaque_tid();
#pragma unroll
            for (int u = 0; u < RPL; ++u) {
                const uint32_t r = ot + u * NT;
                if (r < n) {
#pragma unroll
                    for (int w = 0; w < WI; ++w) rows[r * WI + w] = v[u][w];
                    if constexpr (PRUNE) psig[r] = parent_sig(fd[u], f[u]);
                }
            }
        }
        for (int b = tid; b < C::NB; b += NT) hist[b] = 0;
        EH_STAMP(1);
        // B + C. next bucket: run table, slot map, row loads in flight
        const int bn = bk + G;
        uint32_t nn = 0;
        if (bn < nbk) { // uniform
            nn = rt_commit(pb ^ 1);
            EH_STAMP(7);
            rt_fetch(bn + G);
            prefetch(bn, pb ^ 1, nn);
            issue(0, 2);
            EH_STAMP(9);
        }
        const bool more = bn < nbk;
        __syncthreads();
        EH_STAMP(2);

        // global slot (stage STAGE-1) of LDS row r of the current bucket, from its run table
        auto slot_of = [&](uint32_t r) -> uint32_t {
            const uint32_t b = run_of<NS>(rpos[pb], r);
            return b * SSTRIDE + rsrc[pb][b] + (r - rpos[pb][b]);
        };
        // D1. counting sort of the rows by their RB key: sidx = row ids grouped by key,
        //     bend[key] = end of the key's group
        auto key_of = [&](uint32_t i) -> uint32_t { return rows[i * WI] >> (32 - C::RB); };
        for (int k = tid; k < C::NRESTS; k += NT) bend[k] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < n; i += NT) atomicAdd(&bend[key_of(i)], 1u);
        __syncthreads();
        block_exscan<NT, (C::NRESTS + NT - 1) / NT>(bend, C::NRESTS, wsum);
        for (uint32_t i = tid; i < n; i += NT) sidx[atomicAdd(&bend[key_of(i)], 1u)] = (uint16_t)i;
        if (more) issue(2, 3);
        __syncthreads();
        EH_STAMP(3);

        if constexpr (FINAL) {
            // D2 (final round). Candidates are pairs equal on ALL remaining bits: each sorted
            // position scans the rest of its key group (a few rows). No pair list, so a bucket's
            // pair count is not capped (a capped list here silently lost solutions).
            static_assert(WI == 1, "final-round rows are one word");
            for (uint32_t p = tid; p < n; p += NT) {
                const uint32_t i = sidx[p], ri = rows[i], e = bend[ri >> (32 - C::RB)];
                for (uint32_t q = p + 1; q < e; ++q) {
                    const uint32_t j = sidx[q];
                    if (rows[j] != ri) continue;
                    if constexpr (PRUNE) {
                        const uint32_t si = psig[i], sj = psig[j];
                        if ((si >> 16) == (sj >> 16) || (si >> 16) == (sj & 0xffff) || (si & 0xffff) == (sj >> 16) ||
                            (si & 0xffff) == (sj & 0xffff))
                            if (slot_of(i) / C::AREA == slot_of(j) / C::AREA) continue;
                    }
                    const uint32_t c = atomicAdd(&ncand[nonce], 1u);
                    if (c < (uint32_t)C::MAXCAND) cand[(size_t)nonce * C::MAXCAND + c] = pack_tri(d, i, j);
                }
            }
            if (more) issue(3, 4);
        } else {
            // D2. atomic-free pair enumeration. Sorted position p pairs with every later position
            //     of its group: c_p = bend[key] - p - 1 pairs, first pair index offp[p] (exclusive
            //     scan). A mark p at each group's first pair index, spread by an inclusive
            //     max-scan, tells every pair index k its p; q = p + 1 + (k - offp[p]). Pairs live
            //     in registers (MP per lane: up to MP*NT per bucket, above the row capacity:
            //     capped pair lists lost ~9% of the solutions); identical subtrees and pairs that
            //     share a parent are dropped.
            // c_p is capped at 14 so every prefix fits the u16 offsets (a key group of 16+ rows is
            // ~1e-8 likely; it only loses a few pairs)
            for (uint32_t p = tid; p < n; p += NT) offp[p] = (uint16_t)min(bend[key_of(sidx[p])] - p - 1, 14u);
            __syncthreads();
            const uint32_t P = block_exscan<NT, MPR>(offp, (int)n, wsum);
            const uint32_t Pc = min(P, (uint32_t)(MP * NT));
            if (tid == 0 && P > (uint32_t)(MP * NT)) atomicAdd(&pdrop[STAGE], P - MP * NT);
            for (uint32_t k = tid; k < Pc; k += NT) pmark[k] = 0;
            __syncthreads();
            for (uint32_t p = tid; p < n; p += NT) {
                const uint32_t o = offp[p], e = (p + 1 < n) ? offp[p + 1] : P;
                if (e > o && o < Pc) pmark[o] = (uint16_t)p;
            }
            __syncthreads();
            block_maxscan<NT, MP>(pmark, (int)Pc, wsum);
            uint32_t pv[MP], pd[MP];
#pragma unroll
            for (int u = 0; u < MP; ++u) {
                const uint32_t k = tid + u * NT;
                pv[u] = NIL;
                pd[u] = 0;
                if (k < Pc) {
                    const uint32_t p = pmark[k], q = p + 1 + (k - offp[p]);
                    const uint32_t i = sidx[p], j = sidx[q];
                    const uint32_t x0 = rows[i * WI] ^ rows[j * WI];
                    // identical subtrees are dropped; word 0 differs in all but ~2^-21 of the
                    // pairs, so the remaining words are read only when it matches
                    bool keep = x0 != 0;
                    if (!keep) {
#pragma unroll
                        for (int w = 1; w < WI; ++w) keep |= rows[i * WI + w] != rows[j * WI + w];
                    }
                    if constexpr (PRUNE) {
                        const uint32_t si = psig[i], sj = psig[j];
                        if (keep && ((si >> 16) == (sj >> 16) || (si >> 16) == (sj & 0xffff) ||
                                     (si & 0xffff) == (sj >> 16) || (si & 0xffff) == (sj & 0xffff))) {
                            // signature hit (a shared parent, or ~1e-4 by chance): parents are
                            // shared only if both rows were made by the same workgroup
                            if (slot_of(i) / C::AREA == slot_of(j) / C::AREA) keep = false;
                        }
                    }
                    if (keep) {
                        pv[u] = (j << 16) | i;
                        pd[u] = (x0 >> (32 - C::DB)) & (C::NB - 1); // destination bucket
                        atomicAdd(&hist[pd[u]], 1u);
                    }
                }
            }
            if (more) issue(3, 4);
            __syncthreads();
            EH_STAMP(4);
            // D3. output runs by destination bucket: exclusive scan of the counts -> one column
            //     of CNT/OFF; each pair then takes the next slot of its destination's run
            for (int b = tid; b < C::NB; b += NT) cur[b] = hist[b];
            __syncthreads();
            const uint32_t np = block_exscan<NT>(cur, C::NB, wsum);
            for (int b = tid; b < C::NB; b += NT) {
                CNTout[matout + (size_t)b * C::NB + d] = hist[b];
                OFFout[matout + (size_t)b * C::NB + d] = cur[b];
            }
            __syncthreads(); // every OFF column entry is read before cur[] is advanced
            // slot -> pair table in the (now dead) walk/prefetch union
            uint32_t* spair = reinterpret_cast<uint32_t*>(un);
            static_assert(round_un<C>(CAP) >= C::AREA * 4, "slot table fits the union");
#pragma unroll
            for (int u = 0; u < MP; ++u)
                if (pv[u] != NIL) spair[atomicAdd(&cur[pd[u]], 1u)] = pv[u];
            if (more) issue(4, RPL);
            __syncthreads();
            EH_STAMP(5);
            // D4. emit, one lane per output row in slot order (coalesced): XOR, shift one
            //     digit, store
            const auto rsrc_out = __builtin_amdgcn_make_buffer_rsrc(
                Rout + (size_t)nonce * C::ROWS * C::WMAX + (size_t)d * C::AREA * WO, 0, C::AREA * WO * 4, 0x00020000);
            uint32_t* farea = Fout + (size_t)nonce * C::ROWS + (size_t)d * C::AREA;
            for (uint32_t t = tid; t < np; t += NT) {
                const uint32_t pr = spair[t];
                const uint32_t i = pr & 0xffff, j = pr >> 16;
                uint32_t x[WI + 1], o[WO];
#pragma unroll
                for (int w = 0; w < WI; ++w) x[w] = rows[i * WI + w] ^ rows[j * WI + w];
                x[WI] = 0;
#pragma unroll
                for (int w = 0; w < WO; ++w) o[w] = (x[w] << C::DB) | (x[w + 1] >> (32 - C::DB));
                row_store<WO>(rsrc_out, t * (WO * 4), o);
                farea[t] = pr;
            }
        }
        if constexpr (FINAL) {
            if (more) issue(4, RPL);
        }
        if (more) write_map();
        __syncthreads();
        EH_STAMP(6);
        if (bn >= nbk) break;
        bk = bn;
        n = nn;
        pb ^= 1;
    }
}


// ------------------------------------------------------------------ tree expansion
// F: K arrays of per-stage references; M: K gather maps (M_s for round s at index s-1).
template <class C>
__global__ __launch_bounds__(C::L < 64 ? 64 : C::L) void eh_expand(const uint32_t* __restrict__ F,
                                                                  const uint32_t* __restrict__ M,
                                                                  const uint32_t* __restrict__ ncand,
                                                                  const uint64_t* __restrict__ cand, int batch,
                                                                  uint32_t* __restrict__ out_idx,
                                                                  uint32_t* __restrict__ out_valid) {
    constexpr int L = C::L;
    __shared__ uint32_t buf[2][L];
    __shared__ uint64_t tri[L / 2 > 0 ? L / 2 : 1];
    __shared__ uint32_t dup;
    const uint32_t c = blockIdx.x % C::MAXCAND;
    const uint32_t nonce = blockIdx.x / C::MAXCAND;
    const uint32_t t = threadIdx.x;
    const uint32_t nc = min(ncand[nonce], (uint32_t)C::MAXCAND);
    if (c >= nc) return; // uniform per workgroup
    if (t == 0) {
        tri[0] = cand[(size_t)nonce * C::MAXCAND + c];
        dup = 0;
    }
    int cur = 0;
    // level s: 2^(K-s) triples of round s -> 2^(K-s+1) stage-(s-1) slots
    for (int s = C::K; s >= 1; --s) {
        __syncthreads();
        const uint32_t cnt = 1u << (C::K - s);
        const uint32_t* Ms = M + (size_t)(s - 1) * batch * C::ROWS + (size_t)nonce * C::ROWS;
        if (t < 2 * cnt) {
            const uint64_t tr = tri[t >> 1];
            const uint32_t dd = (uint32_t)(tr >> 32);
            const uint32_t r = (t & 1) ? (((uint32_t)tr >> 16) & 0xffff) : ((uint32_t)tr & 0xffff);
            buf[cur][t] = Ms[(size_t)dd * C::AREA + r];
        }
        __syncthreads();
        if (s > 1 && t < 2 * cnt) {
            const uint32_t slot = buf[cur][t];
            const uint32_t fr = F[(size_t)(s - 1) * batch * C::ROWS + (size_t)nonce * C::ROWS + slot];
            tri[t] = pack_tri(slot / C::AREA, fr & 0xffff, fr >> 16);
        }
    }
    __syncthreads();
    if (t < (uint32_t)L) buf[cur][t] = F[(size_t)nonce * C::ROWS + buf[cur][t]];
    // Canonical order: at each level the subtree with the smaller first index goes left.
    for (int l = 0; l < C::K; ++l) {
        __syncthreads();
        if (t < (uint32_t)L) {
            const uint32_t w = 1u << l;
            const uint32_t j = t & ~(2 * w - 1);
            const bool swap = buf[cur][j + w] < buf[cur][j];
            const uint32_t pos = t - j;
            const uint32_t np = swap ? (pos < w ? pos + w : pos - w) : pos;
            buf[cur ^ 1][j + np] = buf[cur][t];
        }
        cur ^= 1;
    }
    __syncthreads();
    if (t < (uint32_t)L) out_idx[((size_t)nonce * C::MAXCAND + c) * L + t] = buf[cur][t];
    // Distinctness: bitonic sort a copy, then compare neighbours.
    const int o = cur ^ 1;
    if (t < (uint32_t)L) buf[o][t] = buf[cur][t];
    for (uint32_t k = 2; k <= (uint32_t)L; k <<= 1) {
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            __syncthreads();
            if (t < (uint32_t)L) {
                const uint32_t ixj = t ^ jj;
                if (ixj > t) {
                    const uint32_t a = buf[o][t], bb = buf[o][ixj];
                    const bool up = (t & k) == 0;
                    if ((a > bb) == up) {
                        buf[o][t] = bb;
                        buf[o][ixj] = a;
                    }
                }
            }
        }
    }
    __syncthreads();
    if (t + 1 < (uint32_t)L && buf[o][t] == buf[o][t + 1]) atomicOr(&dup, 1u);
    __syncthreads();
    if (t == 0) out_valid[nonce * C::MAXCAND + c] = dup ? 0u : 1u;
}

} // namespace bcpk

namespace bcp {
namespace gpu {

static_assert(sizeof(EhBaseState) == sizeof(bcpk::EhBaseState), "EhBaseState mirror");

EhBaseState MakeEhBaseState(const CBlake2b& st_in) {
    CBlake2b st = st_in;
    Blake2bState& s = st.MutableState();
    if (s.buflen == 128) { // flush a full buffered block as non-final
        s.t[0] += 128;
        if (s.t[0] < 128) s.t[1]++;
        CBlake2b::Compress(s.h, s.buf, s.t[0], s.t[1], false);
        s.buflen = 0;
    }
    if (s.buflen + 4 > 128) throw std::runtime_error("MakeEhBaseState: g would straddle a block boundary");
    if (s.t[1] != 0) throw std::runtime_error("MakeEhBaseState: input too long");
    EhBaseState bs;
    memset(&bs, 0, sizeof(bs));
    memcpy(bs.h, s.h, sizeof(bs.h));
    unsigned char block[128] = {0};
    memcpy(block, s.buf, s.buflen);
    for (int i = 0; i < 16; ++i) memcpy(&bs.m[i], block + 8 * i, 8);
    bs.t0 = s.t[0] + s.buflen + 4;
    bs.g_byte = s.buflen;
    bs.outlen = s.outlen;
    return bs;
}

struct EquihashGpuSolver::Impl {
    unsigned n, k;
    int batch, device;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    DevBuf<bcpk::EhBaseState> d_states;
    DevBuf<uint32_t> d_rows[2], d_cnt[2], d_off[2], d_maps, d_ncand, d_idx, d_valid;
    DevBuf<uint32_t> d_refs, d_pdrop;
    HostBuf<uint32_t> h_pdrop;
    DevBuf<uint64_t> d_cand;
    HostBuf<bcpk::EhBaseState> h_states;
    HostBuf<uint32_t> h_ncand, h_idx, h_valid, h_cnt_sample, h_cnt0;
    size_t genwg = 0;
    size_t rows = 0, L = 0, maxcand = 0, nb = 0, kstages = 0;
    std::vector<size_t> caps; // caps[s]: LDS capacity of the round that reads stage-s rows
    int inflight = 0;
    int ncu = 1;
    bool debug = false, stamp_mode = false;
    DevBuf<uint64_t> d_stamps;
    EhGpuStats stats;
    size_t bytes = 0;

    template <class C> void alloc() {
        rows = C::ROWS;
        L = C::L;
        maxcand = C::MAXCAND;
        nb = C::NB;
        caps.clear();
        for (int r = 1; r <= C::K; ++r) caps.push_back(C::cap(r));
        kstages = C::K;
        d_states.alloc(batch);
        h_states.alloc(batch);
        for (int p = 0; p < 2; ++p) {
            d_rows[p].alloc((size_t)batch * C::ROWS * C::WMAX);
            const size_t m = (size_t)C::NB * std::max(C::NB, C::GENWG);
            d_cnt[p].alloc((size_t)batch * m);
            d_off[p].alloc((size_t)batch * m);
        }
        d_refs.alloc((size_t)C::K * batch * C::ROWS);
        d_maps.alloc((size_t)C::K * batch * C::ROWS);
        d_ncand.alloc(batch);
        d_pdrop.alloc(C::K + 1);
        h_pdrop.alloc(C::K + 1);
        d_cand.alloc((size_t)batch * C::MAXCAND);
        d_idx.alloc((size_t)batch * C::MAXCAND * C::L);
        d_valid.alloc((size_t)batch * C::MAXCAND);
        h_ncand.alloc(batch);
        h_idx.alloc((size_t)batch * C::MAXCAND * C::L);
        h_valid.alloc((size_t)batch * C::MAXCAND);
        h_cnt_sample.alloc((size_t)C::K * C::NB * C::NB);
        h_cnt0.alloc((size_t)C::NB * C::GENWG);
        d_stamps.alloc((size_t)C::K * batch * C::NB * 16);
        genwg = C::GENWG;
        bytes = 2 * d_rows[0].n * 4 + d_refs.n * 4 + d_maps.n * 4 + 4 * d_cnt[0].n * 4 + d_idx.n * 4;
    }

    // Persistent round kernels: as many workgroups as fit on the device at once.
    template <class C, int S, bool ST> int round_grid(int nbk) {
        static int per_cu = -1;
        if (per_cu < 0) {
            int occ = 0;
            BCP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, bcpk::eh_round<C, S, ST>, C::NT, 0));
            per_cu = std::max(occ, 1);
        }
        return std::min(nbk, ncu * per_cu);
    }
    template <class C, int S> void launch_round(int nstates) {
        const int pi = (S - 1) & 1, po = S & 1;
        const uint32_t* fin = d_refs.p + (size_t)(S - 1) * batch * C::ROWS;
        uint32_t* fout = (S < C::K) ? d_refs.p + (size_t)S * batch * C::ROWS : nullptr;
        uint32_t* mout = d_maps.p + (size_t)(S - 1) * batch * C::ROWS;
        const int nbk = C::NB * nstates;
        if (stamp_mode) {
            uint64_t* st = d_stamps.p + (size_t)(S - 1) * batch * C::NB * 16;
            hipLaunchKernelGGL((bcpk::eh_round<C, S, true>), dim3(round_grid<C, S, true>(nbk)), dim3(C::NT), 0,
                               stream, d_rows[pi].p, fin, d_cnt[pi].p, d_off[pi].p, d_rows[po].p, fout, d_cnt[po].p,
                               d_off[po].p, mout, d_ncand.p, d_cand.p, st, d_pdrop.p, nbk);
        } else {
            hipLaunchKernelGGL((bcpk::eh_round<C, S, false>), dim3(round_grid<C, S, false>(nbk)), dim3(C::NT), 0,
                               stream, d_rows[pi].p, fin, d_cnt[pi].p, d_off[pi].p, d_rows[po].p, fout, d_cnt[po].p,
                               d_off[po].p, mout, d_ncand.p, d_cand.p, nullptr, d_pdrop.p, nbk);
        }
        if (debug && S < C::K)
            BCP_HIP_CHECK(hipMemcpyAsync(h_cnt_sample.p + (size_t)S * C::NB * C::NB, d_cnt[po].p,
                                         (size_t)C::NB * C::NB * 4, hipMemcpyDeviceToHost, stream));
    }
    template <class C, int... S> void launch_rounds(int nstates, std::integer_sequence<int, S...>) {
        (launch_round<C, S + 1>(nstates), ...);
    }

    template <class C> void launch(size_t nstates) {
        BCP_HIP_CHECK(hipMemcpyAsync(d_states.p, h_states.p, nstates * sizeof(bcpk::EhBaseState),
                                     hipMemcpyHostToDevice, stream));
        BCP_HIP_CHECK(hipMemsetAsync(d_ncand.p, 0, batch * sizeof(uint32_t), stream));
        BCP_HIP_CHECK(hipMemsetAsync(d_pdrop.p, 0, (C::K + 1) * sizeof(uint32_t), stream));
        if (debug) BCP_HIP_CHECK(hipMemsetAsync(d_refs.p, 0xff, d_refs.n * sizeof(uint32_t), stream));
        BCP_HIP_CHECK(hipEventRecord(ev0, stream));
        // header-shaped inputs (140 B: g lands at byte 12 of the final block) take the
        // zero-message-word BLAKE2b specialisation
        bool hdr = true;
        for (size_t i = 0; i < nstates; ++i) {
            const bcpk::EhBaseState& st = h_states.p[i];
            hdr &= st.g_byte == 12;
            for (int w = 2; w < 16; ++w) hdr &= st.m[w] == 0;
        }
        if (hdr)
            hipLaunchKernelGGL((bcpk::eh_gen<C, true>), dim3(C::GENWG * nstates), dim3(C::NTG), 0, stream,
                               d_states.p, d_rows[0].p, d_refs.p, d_cnt[0].p, d_off[0].p);
        else
            hipLaunchKernelGGL((bcpk::eh_gen<C, false>), dim3(C::GENWG * nstates), dim3(C::NTG), 0, stream,
                               d_states.p, d_rows[0].p, d_refs.p, d_cnt[0].p, d_off[0].p);
        if (debug) { // stage-0 fill per destination bucket, folded to NB x NB-shaped sums on the host
            BCP_HIP_CHECK(hipMemcpyAsync(h_cnt0.p, d_cnt[0].p, (size_t)C::NB * C::GENWG * 4,
                                         hipMemcpyDeviceToHost, stream));
        }
        launch_rounds<C>((int)nstates, std::make_integer_sequence<int, C::K>{});
        constexpr int EB = C::L < 64 ? 64 : C::L;
        hipLaunchKernelGGL((bcpk::eh_expand<C>), dim3(C::MAXCAND * nstates), dim3(EB), 0, stream, d_refs.p,
                           d_maps.p, d_ncand.p, d_cand.p, batch, d_idx.p, d_valid.p);
        BCP_HIP_CHECK(hipGetLastError());
        BCP_HIP_CHECK(hipEventRecord(ev1, stream));
        BCP_HIP_CHECK(
            hipMemcpyAsync(h_ncand.p, d_ncand.p, nstates * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        if (debug)
            BCP_HIP_CHECK(hipMemcpyAsync(h_pdrop.p, d_pdrop.p, (C::K + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                         stream));
        BCP_HIP_CHECK(hipMemcpyAsync(h_valid.p, d_valid.p, nstates * C::MAXCAND * sizeof(uint32_t),
                                     hipMemcpyDeviceToHost, stream));
        BCP_HIP_CHECK(hipMemcpyAsync(h_idx.p, d_idx.p, nstates * C::MAXCAND * C::L * sizeof(uint32_t),
                                     hipMemcpyDeviceToHost, stream));
    }
};

template <class F> static void dispatch_cfg(unsigned n, unsigned k, F&& f) {
    if (n == 200 && k == 9) f(bcpk::Cfg200_9{});
    else if (n == 96 && k == 5) f(bcpk::Cfg96_5{});
    else if (n == 48 && k == 5) f(bcpk::Cfg48_5{});
    else throw std::invalid_argument("EquihashGpuSolver: unsupported (N,K); GPU supports (200,9),(96,5),(48,5)");
}

EquihashGpuSolver::EquihashGpuSolver(unsigned n, unsigned k, int batch, int device) : impl(new Impl) {
    if (batch < 1) throw std::invalid_argument("batch must be >= 1");
    impl->n = n;
    impl->k = k;
    impl->batch = batch;
    impl->device = UseDevice(device);
    BCP_HIP_CHECK(hipDeviceGetAttribute(&impl->ncu, hipDeviceAttributeMultiprocessorCount, impl->device));
    BCP_HIP_CHECK(hipStreamCreateWithFlags(&impl->stream, hipStreamNonBlocking));
    BCP_HIP_CHECK(hipEventCreate(&impl->ev0));
    BCP_HIP_CHECK(hipEventCreate(&impl->ev1));
    dispatch_cfg(n, k, [&](auto c) { impl->alloc<decltype(c)>(); });
}

EquihashGpuSolver::~EquihashGpuSolver() {
    if (impl) {
        (void)hipSetDevice(impl->device);
        if (impl->stream) (void)hipStreamSynchronize(impl->stream);
        if (impl->ev0) (void)hipEventDestroy(impl->ev0);
        if (impl->ev1) (void)hipEventDestroy(impl->ev1);
        if (impl->stream) (void)hipStreamDestroy(impl->stream);
    }
}

unsigned EquihashGpuSolver::N() const { return impl->n; }
unsigned EquihashGpuSolver::K() const { return impl->k; }
int EquihashGpuSolver::Batch() const { return impl->batch; }
const EhGpuStats& EquihashGpuSolver::Stats() const { return impl->stats; }
void EquihashGpuSolver::SetDebug(bool on) { impl->debug = on; }
void EquihashGpuSolver::SetStampMode(bool on) { impl->stamp_mode = on; }

// Mean cycles per phase per round (diagnostic stamp builds): [stage][phase delta].
std::vector<std::vector<double>> EquihashGpuSolver::PhaseCycles(int nonces) {
    BCP_HIP_CHECK(hipSetDevice(impl->device));
    BCP_HIP_CHECK(hipStreamSynchronize(impl->stream));
    const size_t per = (size_t)impl->batch * impl->nb * 16;
    std::vector<uint64_t> h(impl->kstages * per);
    BCP_HIP_CHECK(hipMemcpy(h.data(), impl->d_stamps.p, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<std::vector<double>> out;
    for (size_t s = 0; s < impl->kstages; ++s) {
        std::vector<double> acc(10, 0.0);
        size_t cnt = 0;
        for (size_t wg = 0; wg < (size_t)nonces * impl->nb; ++wg) {
            const uint64_t* t = &h[s * per + wg * 16];
            if (t[0] == 0) continue;
            for (int k = 1; k < 7; ++k)
                if (t[k] >= t[k - 1] && t[k] != 0) acc[k] += (double)(t[k] - t[k - 1]);
            acc[0] += (double)((t[6] ? t[6] : t[3]) - t[0]);
            // prefetch split: run-table commit | slot map | M map + load issue | barrier
            if (t[7] && t[8] && t[9] && t[7] >= t[1] && t[8] >= t[7] && t[9] >= t[8] && t[2] >= t[9]) {
                acc[7] += (double)(t[7] - t[1]);
                acc[8] += (double)(t[8] - t[7]);
                acc[9] += (double)(t[9] - t[8]);
            }
            ++cnt;
        }
        for (auto& a : acc) a = cnt ? a / cnt : 0;
        out.push_back(acc);
    }
    return out;
}
void EquihashGpuSolver::ResetStats() { impl->stats = EhGpuStats(); }

// Debug: parent refs F (K stages) then gather maps M (K rounds) of nonce 0 of the last batch,
// each ROWS slots; with SetDebug(true) never-written F slots read 0xffffffff.
std::vector<uint32_t> EquihashGpuSolver::DebugDump() {
    BCP_HIP_CHECK(hipSetDevice(impl->device));
    BCP_HIP_CHECK(hipStreamSynchronize(impl->stream));
    const size_t R = impl->rows, K = impl->kstages, B = impl->batch;
    std::vector<uint32_t> out(2 * K * R);
    for (size_t s = 0; s < K; ++s) {
        BCP_HIP_CHECK(hipMemcpy(out.data() + s * R, impl->d_refs.p + s * B * R, R * 4, hipMemcpyDeviceToHost));
        BCP_HIP_CHECK(hipMemcpy(out.data() + (K + s) * R, impl->d_maps.p + s * B * R, R * 4, hipMemcpyDeviceToHost));
    }
    return out;
}
size_t EquihashGpuSolver::DeviceBytes() const { return impl->bytes; }

void EquihashGpuSolver::Launch(const std::vector<EhBaseState>& states) {
    if (states.empty() || (int)states.size() > impl->batch) throw std::invalid_argument("bad number of states");
    if (impl->inflight) throw std::runtime_error("EquihashGpuSolver: Collect() the previous launch first");
    BCP_HIP_CHECK(hipSetDevice(impl->device));
    memcpy(impl->h_states.p, states.data(), states.size() * sizeof(EhBaseState));
    dispatch_cfg(impl->n, impl->k, [&](auto c) { impl->launch<decltype(c)>(states.size()); });
    impl->inflight = (int)states.size();
}

std::vector<std::vector<std::vector<uint32_t>>> EquihashGpuSolver::Collect() {
    if (!impl->inflight) throw std::runtime_error("EquihashGpuSolver: nothing in flight");
    BCP_HIP_CHECK(hipSetDevice(impl->device));
    BCP_HIP_CHECK(hipStreamSynchronize(impl->stream));
    const int ns = impl->inflight;
    impl->inflight = 0;
    float ms = 0;
    BCP_HIP_CHECK(hipEventElapsedTime(&ms, impl->ev0, impl->ev1));
    impl->stats.gpu_ms += ms;
    impl->stats.nonces += ns;
    if (impl->debug) {
        // nonce 0: per stage, rows offered to each destination bucket vs its LDS capacity
        const size_t NB = impl->nb;
        impl->stats.stage_rows.assign(impl->kstages, 0);
        impl->stats.stage_dropped.assign(impl->kstages, 0);
        impl->stats.stage_maxfill.assign(impl->kstages, 0);
        impl->stats.stage_top.assign(impl->kstages, {});
        impl->stats.pair_dropped.assign(impl->h_pdrop.p, impl->h_pdrop.p + impl->kstages + 1);
        for (size_t s = 0; s < impl->kstages; ++s) {
            const size_t ns = s == 0 ? impl->genwg : NB;
            const uint32_t* m = s == 0 ? impl->h_cnt0.p : impl->h_cnt_sample.p + s * NB * NB;
            std::vector<uint64_t> fills;
            for (size_t dd = 0; dd < NB; ++dd) {
                uint64_t fill = 0;
                for (size_t src = 0; src < ns; ++src) fill += m[dd * ns + src];
                fills.push_back(fill);
                impl->stats.stage_rows[s] += fill;
                impl->stats.stage_maxfill[s] = std::max<uint64_t>(impl->stats.stage_maxfill[s], fill);
                if (fill > impl->caps[s]) {
                    impl->stats.stage_dropped[s] += fill - impl->caps[s];
                    impl->stats.dropped_rows += fill - impl->caps[s];
                }
            }
            std::sort(fills.rbegin(), fills.rend());
            fills.resize(std::min<size_t>(fills.size(), 8));
            impl->stats.stage_top[s] = fills;
        }
    }
    std::vector<std::vector<std::vector<uint32_t>>> out(ns);
    if (impl->debug) {
        impl->stats.debug_cands.clear();
        const uint32_t nc = std::min<uint32_t>(impl->h_ncand.p[0], (uint32_t)impl->maxcand);
        for (uint32_t c = 0; c < nc; ++c) {
            const uint32_t* p = impl->h_idx.p + (size_t)c * impl->L;
            impl->stats.debug_cands.emplace_back(p, p + impl->L);
        }
    }
    for (int nn = 0; nn < ns; ++nn) {
        uint32_t nc = std::min<uint32_t>(impl->h_ncand.p[nn], (uint32_t)impl->maxcand);
        impl->stats.candidates += nc;
        for (uint32_t c = 0; c < nc; ++c) {
            if (!impl->h_valid.p[nn * impl->maxcand + c]) {
                impl->stats.duplicates++;
                continue;
            }
            const uint32_t* p = impl->h_idx.p + ((size_t)nn * impl->maxcand + c) * impl->L;
            std::vector<uint32_t> v(p, p + impl->L);
            bool seen = false;
            for (auto& prev : out[nn]) seen |= (prev == v);
            if (seen) continue;
            out[nn].push_back(std::move(v));
            impl->stats.solutions++;
        }
    }
    return out;
}

std::vector<std::vector<std::vector<uint32_t>>> EquihashGpuSolver::Solve(const std::vector<EhBaseState>& states) {
    Launch(states);
    return Collect();
}

} // namespace gpu
} // namespace bcp
