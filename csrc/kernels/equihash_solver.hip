// Equihash solver for CDNA4 (gfx950) — the GPU replacement for the reference's
// CPU BasicSolve/OptimisedSolve (reference src/crypto/equihash.cpp:332-722,
// called from generateBlocks src/rpc/mining.cpp:161-199).
//
// Design: a bucket-sorted Wagner solver with parent pointers and contiguous buckets.
//
//  * Rows are bucketed on the top BB bits of the current digit (NB = 2^BB buckets, ~INIT/NB rows
//    each). (200,9) runs BB = 9: 512 buckets of ~4096 rows, one 1024-thread round workgroup per
//    CU (145 KiB of LDS). 1024 buckets of ~2048 rows with two 512-thread workgroups (<= 80 KiB
//    each) per CU measured slower (the phases are latency-bound per lane, and the producer runs
//    are 4x shorter), profiles/equihash_r4.md.
//    Every stage keeps each bucket CONTIGUOUS in its own area of AREA row slots.
//  * Every kernel works "one workgroup per bucket". A producer workgroup counting-sorts its
//    output rows by destination bucket in LDS, then claims one run per destination with ONE
//    device-scope atomicAdd on that bucket's fill counter (issued as soon as the histogram is
//    known so its latency hides behind the scan and scatter), and writes its rows into the
//    claimed runs. The consumer round then reads its bucket as one contiguous block (16-byte
//    loads, straight into LDS): no run tables, slot maps or per-row gather maps.
//  * Collisions on the remaining RB = DB-BB bits of the digit are found by a counting sort of
//    the bucket on those bits and an atomic-free pair enumeration (scan + max-scan); each output
//    row keeps a parent triple (producing bucket, LDS row i, LDS row j), so nothing ever carries
//    index lists: the parents of a stage-s row are the stage-(s-1) slots bucket*AREA + i and
//    bucket*AREA + j.
//  * Depth-1 duplicate pruning (pairs whose rows share a parent are dropped) wherever the parent
//    words fit in the round's LDS budget.
//  * Final round: pairs equal on all remaining bits are candidates; eh_expand walks the K levels
//    of parent triples, canonicalises subtree order (reference IsValidSolution ordering rule)
//    and rejects repeated indices (LDS bitonic sort).
//  * Block scans use DPP row shifts/broadcasts inside a wave and one LDS word per wave
//    across waves: two barriers per scan, no ds_bpermute traffic.
//
// Memory layout: every stage has its own slot array and a stage-s slot holds the row followed by
// its parent word(s), so the emit writes one contiguous slot per output row and a pruning round
// gets the parents with the rows. Keeping all K stage arrays costs ~50 words per slot per nonce
// (≈17 GB per 32-nonce solver, against 288 GB of HBM); the parents must outlive the rows anyway
// for the final expansion. Per row per round: one contiguous slot read, one slot write into a
// claimed run.
#include <hip/hip_runtime.h>

#include "crypto/hashes.h"
#include "kernels/blake2b_device.h"
#include "kernels/gpu_api.h"
#include "kernels/hip_util.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <utility>

// Build options (each either the measured default or covered by the GPU tests; the variants that
// were measured and rejected in rounds 3-5 are at git tag solver-r5-knobs, profiles/equihash_r4.md
// and profiles/equihash_r5.md):
#ifndef BCP_EH_XCD_MAP // 1: every kernel of a nonce runs on one XCD (nonce % 8), so the run writes
#define BCP_EH_XCD_MAP 1  //    of a nonce meet in one L2 (batches that are a multiple of 8 nonces)
#endif
#ifndef BCP_EH_PF_SLICES // the next bucket's rows are prefetched in this many slices
#define BCP_EH_PF_SLICES 3
#endif
#ifndef BCP_EH_GEN_HPT // (200,9) register generation: hashes per thread
#define BCP_EH_GEN_HPT 2
#endif
#ifndef BCP_EH_GEN_NT // (200,9) register generation: threads per workgroup
#define BCP_EH_GEN_NT 512
#endif
#ifndef BCP_EH_PRUNE_FROM // first round that drops pairs sharing a parent (reads the parent words with the rows);
                          // the final round always does.
#define BCP_EH_PRUNE_FROM 9 //  9 = the final round only: +4.2% Sol/s over 2 at the same recall (profiles/equihash_r5.md)
#endif
#ifndef BCP_EH_MP_LATE // extra pair slots per lane in the late collision rounds (see round_mp)
#define BCP_EH_MP_LATE 1
#endif
#ifndef BCP_EH_MP_LATE_FROM
#define BCP_EH_MP_LATE_FROM 8
#endif

namespace bcpk {

// N, K: Equihash parameters. BB: bucket bits. CAP/CAP4/CAP3: LDS row capacity of rounds reading
// rows of >= 5, 4, <= 3 words. NT: threads per round workgroup; WGCU: round workgroups per CU
// the LDS budget must allow. GENWG/NTG: LDS-sorted generation geometry; GNT x GHPT: register
// generation (threads x hashes per thread; 0 = use the LDS-sorted kernel).
template <int N_, int K_, int BB_, int CAP_, int NT_, int GENWG_, int NTG_, int MAXCAND_, int CAP4_ = CAP_,
          int CAP3_ = CAP_, int WGCU_ = 1, int GNT_ = 512, int GHPT_ = 2, int CAPF_ = 0, int MPX_ = 0>
struct EhCfg {
    static constexpr int N = N_, K = K_;
    static constexpr int DB = N / (K + 1);           // digit bits
    static constexpr int BB = BB_;                   // bucket bits
    static constexpr int RB = DB - BB_;              // in-bucket collision bits
    static constexpr int NB = 1 << BB_;              // buckets (= areas of every stage)
    static constexpr int NRESTS = 1 << RB;
    // LDS row capacity of a round by the width of the rows it reads: the narrow late rounds
    // hold more rows (their buckets and pair lists overflow most, from duplicate subtrees)
    static constexpr int CAP = CAP_;                 // rounds reading >= 5-word rows
    // CAPF: the final round's capacity (0 = CAP3). Without depth-1 pruning before the final round,
    // duplicate subtrees pile up in a few stage-(K-1) buckets; a larger final area keeps the valid
    // rows of such a bucket from being crowded out (which rows are dropped follows the atomics).
    static constexpr int CAPF = CAPF_ > 0 ? CAPF_ : CAP3_;
    static constexpr int MPX = MPX_;                 // extra pair-list slots per lane in every collision round
    static constexpr int cap(int round) {
        return round == K_ ? CAPF : words(round - 1) >= 5 ? CAP_ : words(round - 1) == 4 ? CAP4_ : CAP3_;
    }
    // largest non-final capacity (sizes the per-lane pair registers) and the area of every stage
    static constexpr int AREA_NF = CAP_ > CAP4_ ? (CAP_ > CAP3_ ? CAP_ : CAP3_) : (CAP4_ > CAP3_ ? CAP4_ : CAP3_);
    static constexpr int AREA = AREA_NF > CAPF ? AREA_NF : CAPF;
    static constexpr int NT = NT_;                   // threads per round workgroup
    static constexpr int NW = NT_ / 64;
    static constexpr int WGCU = WGCU_;
    static constexpr int LDS_BUDGET = 160 * 1024 / WGCU_;
    static constexpr int INIT = 1 << (DB + 1);
    static constexpr int GENWG = GENWG_;             // LDS-sorted generation: workgroups per nonce
    static constexpr int NTG = NTG_;                 // LDS-sorted generation: threads per workgroup
    static constexpr int GNT = GNT_, GHPT = GHPT_;   // register generation geometry
    static constexpr int RPW = INIT / GENWG_;        // rows per generation workgroup
    static constexpr int IPH = 512 / N;
    static constexpr int NBYTES = N / 8;
    static constexpr int MAXCAND = MAXCAND_;
    static constexpr int L = 1 << K;
    static constexpr int bits(int stage) { return N - stage * DB - BB_; }
    static constexpr int words(int stage) { return (bits(stage) + 31) / 32; }
    static constexpr int WMAX = words(0);
    // Compact parents: the triple (d, i, j) as ONE word. i and j take IB bits each in the two
    // halves of the word, the 16 - IB spare bits of each half carry DX bits of d, and the DR
    // remaining bits of d ride in the low (padding) bits of the row's last word.
    static constexpr int IB = AREA <= 4096 ? 12 : 13;
    static constexpr int DH = 16 - IB;
    static constexpr uint32_t DHM = (1u << DH) - 1;
    static constexpr int DX = 2 * DH;
    static constexpr int DR = BB_ > DX ? BB_ - DX : 0;
    static constexpr uint32_t RMASK = (1u << DR) - 1;
    static constexpr uint32_t IMASK = ((1u << IB) - 1) * 0x10001u;
    static constexpr bool cp(int stage) {
        return stage >= 1 && stage < K && 32 * words(stage) - bits(stage) >= DR;
    }
    static constexpr uint32_t rmask(int stage) { return cp(stage) ? RMASK : 0u; } // parent bits in a row's padding
    // words per slot of stage s: the row, plus (s >= 1) its parent word(s)
    static constexpr int sw(int stage) { return stage == 0 ? words(0) : words(stage) + (cp(stage) ? 1 : 2); }
    static constexpr size_t ROWS = (size_t)NB * AREA; // slots per stage per nonce
    // 16-bit LDS histograms (two counters per word) where 32-bit ones would not fit two per CU
    static constexpr bool H16 = NB > 512;
    static constexpr int HW = H16 ? NB / 2 : NB;      // words per histogram
    static_assert(RPW * GENWG_ == INIT && RPW < 65535, "generation split");
    static_assert(RB > 0 && DB < 32, "digit geometry");
    static_assert(AREA < (1 << IB), "LDS row indices in parent words and signatures");
    static_assert(NT_ % 64 == 0 && NT_ <= 1024 && (NB <= NT_ || NB % NT_ == 0) && NB <= NTG_ && NT_ / 64 <= 64,
                  "workgroup shape");
    static_assert(words(K - 1) == 1, "final round keeps whole rows in one LDS word");
};

// Mainnet/testnet (200,9): 512 buckets x ~4096 rows, one 1024-thread round workgroup per CU;
// (96,5); regtest (48,5).
#ifndef BCP_EH_CAPF // (200,9) final-round capacity (rows per bucket; the stage areas grow to match)
#define BCP_EH_CAPF 6016 // 5120 overflowed by 2-140 rows in ~12 buckets per 32 nonces (recall_base.json, round 5); 6016 keeps two final-round WGs per CU
#endif
using Cfg200_9 = EhCfg<200, 9, 9, 4416, 1024, 512, 1024, 256, 4864, 5120, 1, BCP_EH_GEN_NT, BCP_EH_GEN_HPT, BCP_EH_CAPF>;
// (96,5): one extra pair slot per lane. ~1024 rows per bucket over 512 keys make ~1024 pairs, and
// a list of 1280 overflowed in some bucket of most nonces: 84 + 18 + 36 + ~80 pairs per 16 nonces
// in rounds 1-4, which pairs depending on the atomics' order, so a solution was lost now and then
// (tools/eh_crosscheck.py --n 96 --k 5, profiles/equihash_r6.md).
using Cfg96_5 = EhCfg<96, 5, 7, 1280, 256, 256, 256, 256, 1280, 1280, 1, 512, 2, 0, 1>;
using Cfg48_5 = EhCfg<48, 5, 3, 512, 64, 8, 64, 256>; // 512-slot areas: 8 pairs per lane (a 256-pair list overflowed on duplicate-heavy nonces)

constexpr uint32_t NIL = 0xffffffffu;
constexpr uint32_t OOB = 0x80000000u; // buffer offset past every descriptor's range: access dropped
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
typedef uint32_t u3v __attribute__((ext_vector_type(3)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ wave / block scans
// DPP controls (GFX9 encoding): row_shr:n = 0x110|n, row_bcast:15 = 0x142, row_bcast:31 = 0x143,
// wave_shr:1 = 0x138. Lanes whose source is outside the row / disabled keep `old` (= 0, the
// identity of both + and max over unsigned values). All lanes of the wave must be active.
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xf, false);
}
// Inclusive wave-wide sum (MAX = false) or max (MAX = true).
template <bool MAX> __device__ __forceinline__ uint32_t wave_incl(uint32_t x) {
    auto op = [](uint32_t a, uint32_t b) -> uint32_t { return MAX ? (a > b ? a : b) : a + b; };
    x = op(x, dpp0<0x111>(x));
    x = op(x, dpp0<0x112>(x));
    x = op(x, dpp0<0x114>(x));
    x = op(x, dpp0<0x118>(x));
    x = op(x, dpp0<0x142, 0xa>(x));
    x = op(x, dpp0<0x143, 0xc>(x));
    return x;
}

// Block-wide exclusive sum over n (<= MAXPER*NT) values: src[i] -> dst[i] (src may be dst);
// thread t owns `per` consecutive entries. Wave totals go through `wsum` (>= NT/64 entries);
// every wave combines them itself, so the scan costs two barriers (the second makes dst
// visible and frees wsum). Returns the total; `mine` (optional) receives the exclusive prefix of
// the thread's first entry.
template <int NT, int MAXPER = 4, class TS = uint32_t, class TD = TS>
__device__ uint32_t block_exscan(const TS* src, TD* dst, int n, uint32_t* wsum, uint32_t* mine = nullptr) {
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int per = (n + NT - 1) / NT;
    uint32_t local[MAXPER];
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < MAXPER; ++q) {
        const int i = tid * per + q;
        local[q] = (q < per && i < n) ? (uint32_t)src[i] : 0u;
        s += local[q];
    }
    const uint32_t x = wave_incl<false>(s);
    if (NW > 1) {
        if (lane == 63) wsum[wid] = x;
        __syncthreads();
    }
    const uint32_t wt = (NW > 1 && lane < NW) ? wsum[lane] : 0u;
    const uint32_t ws = wave_incl<false>(wt);
    const uint32_t before = NW > 1 ? __builtin_amdgcn_readlane(ws, wid) - __builtin_amdgcn_readlane(wt, wid) : 0u;
    const uint32_t total = NW > 1 ? __builtin_amdgcn_readlane(ws, NW - 1) : __builtin_amdgcn_readlane(x, 63);
    uint32_t base = before + x - s;
    if (mine) *mine = base;
#pragma unroll
    for (int q = 0; q < MAXPER; ++q) {
        const int i = tid * per + q;
        if (q < per && i < n) dst[i] = (TD)base;
        base += local[q];
    }
    __syncthreads();
    return total;
}
template <int NT, int MAXPER = 4, class T = uint32_t>
__device__ uint32_t block_exscan(T* v, int n, uint32_t* wsum) {
    return block_exscan<NT, MAXPER, T, T>(v, v, n, wsum);
}

// Inclusive prefix maximum in place (entries u32 or u16); two barriers.
template <int NT, int MAXPER = 4, class T = uint32_t>
__device__ void block_maxscan(T* v, int n, uint32_t* wsum) {
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int per = (n + NT - 1) / NT;
    uint32_t local[MAXPER];
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < MAXPER; ++q) {
        const int i = tid * per + q;
        local[q] = (q < per && i < n) ? (uint32_t)v[i] : 0u;
        s = max(s, local[q]);
    }
    const uint32_t x = wave_incl<true>(s);
    const uint32_t excl = dpp0<0x138>(x); // wave_shr:1 -> lane l sees lane l-1 (lane 0: 0)
    if (NW > 1) {
        if (lane == 63) wsum[wid] = x;
        __syncthreads();
    }
    const uint32_t wt = (NW > 1 && lane < NW) ? wsum[lane] : 0u;
    const uint32_t ws = wave_incl<true>(wt);
    const uint32_t before = (NW > 1 && wid > 0) ? __builtin_amdgcn_readlane(ws, wid - 1) : 0u;
    uint32_t run = max(before, excl);
#pragma unroll
    for (int q = 0; q < MAXPER; ++q) {
        const int i = tid * per + q;
        run = max(run, local[q]);
        if (q < per && i < n) v[i] = (T)run;
    }
    __syncthreads();
}

// Row I/O of W dwords at a dword-aligned byte offset through a buffer descriptor: one
// 16-byte access plus a remainder (dword-aligned 16-byte buffer accesses are legal on gfx950).
template <int W> __device__ __forceinline__ void row_store(__amdgpu_buffer_rsrc_t rs, uint32_t off, const uint32_t* v) {
    if constexpr (W >= 4) {
        const u4v x = {v[0], v[1], v[2], v[3]};
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, off, 0, 0);
        row_store<W - 4>(rs, off + 16, v + 4);
    } else if constexpr (W == 3) {
        const u3v x = {v[0], v[1], v[2]};
        __builtin_amdgcn_raw_buffer_store_b96(x, rs, off, 0, 0);
    } else if constexpr (W == 2) {
        const u2v x = {v[0], v[1]};
        __builtin_amdgcn_raw_buffer_store_b64(x, rs, off, 0, 0);
    } else if constexpr (W == 1) {
        __builtin_amdgcn_raw_buffer_store_b32(v[0], rs, off, 0, 0);
    }
}

template <int W> __device__ __forceinline__ void row_load(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t* v) {
    if constexpr (W >= 4) {
        const u4v x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
        v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w;
        row_load<W - 4>(rs, off + 16, v + 4);
    } else if constexpr (W == 3) {
        const u3v x = __builtin_amdgcn_raw_buffer_load_b96(rs, off, 0, 0);
        v[0] = x.x, v[1] = x.y, v[2] = x.z;
    } else if constexpr (W == 2) {
        const u2v x = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
        v[0] = x.x, v[1] = x.y;
    } else if constexpr (W == 1) {
        v[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
    }
}

// x = LDS row i XOR LDS row j (rows of WI words): 8-byte LDS reads when rows are 8-byte aligned
// (even WI). Rows are random here, so every read is bank-conflict bound; a ds_read_b64 spreads its
// lanes over 64 banks where a ds_read2_b32 pays two 32-bank conflict rounds.
template <int WI> __device__ __forceinline__ void lds_row_xor(const uint32_t* rows, uint32_t i, uint32_t j, uint32_t* x) {
    if constexpr (WI % 2 == 0) {
        const u2v* r2 = reinterpret_cast<const u2v*>(rows);
#pragma unroll
        for (int w = 0; w < WI / 2; ++w) {
            const u2v a = r2[i * (WI / 2) + w], b = r2[j * (WI / 2) + w];
            x[2 * w] = a.x ^ b.x;
            x[2 * w + 1] = a.y ^ b.y;
        }
    } else {
#pragma unroll
        for (int w = 0; w < WI; ++w) x[w] = rows[i * WI + w] ^ rows[j * WI + w];
    }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}

// XCD-aware work mapping. Workgroups are dispatched round-robin over the 8 XCDs (workgroup b
// on XCD b % 8), and each XCD has its own L2. A producer writes runs into every destination
// bucket of its nonce; a 128-byte line at a run boundary is shared by two producers. With all
// workgroups of a nonce on the same XCD those partial lines merge in one L2 before they are
// written back (non-temporal stores, which skip the L2 merge, measured 2x slower).
constexpr int NXCD = 8;
// it-th bucket of workgroup b among nbk = NB * nonces buckets (grid G); -1 when done.
template <int NB> __device__ __forceinline__ int xcd_bucket(int b, int it, int G, int nbk) {
    const int nonces = nbk / NB;
    if (!BCP_EH_XCD_MAP || G % NXCD || nonces % NXCD) {
        const int bk = b + it * G;
        return bk < nbk ? bk : -1;
    }
    const int x = b % NXCD, j = b / NXCD + it * (G / NXCD);
    if (j >= NB * (nonces / NXCD)) return -1;
    return (x + NXCD * (j / NB)) * NB + j % NB;
}

// ------------------------------------------------------------------ stage 0
// Generation workgroup gw of a nonce hashes rows [gw*RPW, (gw+1)*RPW), counting-sorts them by
// bucket in LDS, claims one run per destination bucket (device-scope atomicAdd on the stage-0
// fill counters CTR0[nonce][NB]) and writes every row into its run; the leaf index of each
// slot goes to LEAF.
template <class C, bool HDR>
__global__ __launch_bounds__(C::NTG) void eh_gen(const EhBaseState* __restrict__ states, uint32_t* __restrict__ R,
                                                 uint32_t* __restrict__ LEAF, uint32_t* __restrict__ CTR0) {
    constexpr int W0 = C::words(0);
    constexpr int SW = (C::N + 31) / 32 + 1;
    constexpr int NTG = C::NTG;
    constexpr uint32_t OCAP = C::cap(1);
    __shared__ uint32_t rows[C::RPW * W0];
    __shared__ uint16_t dst[C::RPW];
    __shared__ uint16_t perm[C::RPW];
    __shared__ uint32_t hist[C::NB], cur[C::NB], base[C::NB];
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
    // claim the runs; the returned bases are used only after the scan and the scatter
    uint32_t myb = 0, start = 0;
    if (tid < C::NB && hist[tid]) myb = atomicAdd(&CTR0[(size_t)nonce * C::NB + tid], hist[tid]);
    block_exscan<NTG>(hist, cur, C::NB, wsum, &start); // cur = run offsets inside this workgroup's sorted order
    for (int li = tid; li < C::RPW; li += NTG) perm[atomicAdd(&cur[dst[li]], 1u)] = (uint16_t)li;
    if (tid < C::NB) base[tid] = myb - start; // sorted position t of bucket d -> run position base[d] + t
    __syncthreads();
    constexpr int SW0 = C::sw(0);
    const auto rs = buf_rsrc(R + (size_t)nonce * C::ROWS * SW0, (uint32_t)(C::ROWS * SW0 * 4));
    uint32_t* leaf = LEAF + (size_t)nonce * C::ROWS;
    for (int t = tid; t < C::RPW; t += NTG) {
        const uint32_t li = perm[t], d = dst[li];
        const uint32_t pos = base[d] + (uint32_t)t;
        if (pos < OCAP) {
            uint32_t o[W0];
#pragma unroll
            for (int w = 0; w < W0; ++w) o[w] = rows[li * W0 + w];
            const uint32_t slot = d * C::AREA + pos;
            row_store<SW0>(rs, slot * (SW0 * 4), o);
            leaf[slot] = r0 + li;
        }
    }
}

// Register-resident generation for configs whose rows split evenly over hashes (IPH | RPW):
// every thread keeps the HPT*IPH rows it hashed in VGPRs, takes its rank inside this
// workgroup's run of each row's bucket with an LDS atomicAdd (returning), and after the
// run claims writes the rows straight from registers. LDS holds only the two NB-entry
// tables, so several workgroups share a CU and one's hashing (VALU) overlaps another's
// claim and scatter (memory) — the LDS-sorted eh_gen above holds a whole CU with its 118 KB
// row buffer and runs those phases back to back.
template <class C, int NTG, int HPT> struct GenReg {
    static constexpr int RPT = HPT * C::IPH;            // rows per thread
    static constexpr int RPW = NTG > 0 ? NTG * RPT : 1; // rows per workgroup
    static constexpr bool OK = NTG > 0 && C::INIT % RPW == 0;
    static constexpr int GWG = OK ? C::INIT / RPW : 1;  // workgroups per nonce
};
template <class C, bool HDR, int NTG, int HPT>
__global__ __launch_bounds__(NTG) __attribute__((amdgpu_waves_per_eu(1))) void eh_gen_reg(const EhBaseState* __restrict__ states, uint32_t* __restrict__ R,
                                                  uint32_t* __restrict__ LEAF, uint32_t* __restrict__ CTR0, int items) {
    using G = GenReg<C, NTG, HPT>;
    static_assert(G::OK, "register generation geometry");
    constexpr int W0 = C::words(0);
    constexpr int SW = (C::N + 31) / 32 + 1;
    constexpr uint32_t OCAP = C::cap(1);
    __shared__ uint32_t hist[C::NB], base[C::NB];
    __shared__ uint64_t r0p[HDR ? 16 : 1]; // the nonce's g-independent round-0 prefix
    const int tid = threadIdx.x;
    // work item b = (nonce, gw); a persistent grid (gridDim.x < items, a multiple of 8) keeps every
    // item of a workgroup on that workgroup's XCD
    for (int b = blockIdx.x; b < items; b += gridDim.x) {
    int gw = b % G::GWG;
    int nonce = b / G::GWG;
    if (BCP_EH_XCD_MAP && (items / G::GWG) % NXCD == 0 && gridDim.x % NXCD == 0) { // nonce n's workgroups on XCD n % 8
        const int x = b % NXCD, j = b / NXCD;
        gw = j % G::GWG;
        nonce = x + NXCD * (j / G::GWG);
    }
    if (b != (int)blockIdx.x) __syncthreads(); // the previous item's scatter has read base[]
    const EhBaseState& bs = states[nonce];
    for (int i = tid; i < C::NB; i += NTG) hist[i] = 0;
    if constexpr (HDR) {
        if (tid == 0) {
            uint64_t P[16];
            eh_hdr_round0_uniform(bs, P);
#pragma unroll
            for (int i = 0; i < 16; ++i) r0p[i] = P[i];
        }
    }
    __syncthreads();
    const uint32_t r0 = (uint32_t)gw * G::RPW;
    const uint32_t g0 = r0 / C::IPH;
    uint32_t rw[G::RPT][W0];
    uint32_t rk[G::RPT]; // (rank within this workgroup's run << 16) | bucket
#pragma unroll
    for (int hh = 0; hh < HPT; ++hh) {
        const uint32_t g = g0 + hh * NTG + tid;
        uint64_t h[8];
        if constexpr (HDR) {
            uint64_t P[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) P[i] = r0p[i];
            eh_hash_g_hdr_from(P, bs, g, h);
        } else {
            eh_hash_g(bs, g, h);
        }
#pragma unroll
        for (int s = 0; s < C::IPH; ++s) {
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
            const int q = hh * C::IPH + s;
            const uint32_t d = S[0] >> (32 - C::BB);
#pragma unroll
            for (int w = 0; w < W0; ++w) rw[q][w] = (S[w] << C::BB) | (S[w + 1] >> (32 - C::BB));
            rk[q] = (atomicAdd(&hist[d], 1u) << 16) | d;
        }
    }
    __syncthreads();
    // claim one run per destination bucket
    for (int b = tid; b < C::NB; b += NTG) {
        const uint32_t c = hist[b];
        base[b] = c ? atomicAdd(&CTR0[(size_t)nonce * C::NB + b], c) : 0u;
    }
    __syncthreads();
    constexpr int SW0 = C::sw(0);
    const auto rs = buf_rsrc(R + (size_t)nonce * C::ROWS * SW0, (uint32_t)(C::ROWS * SW0 * 4));
    const auto rl = buf_rsrc(LEAF + (size_t)nonce * C::ROWS, (uint32_t)(C::ROWS * 4));
#pragma unroll
    for (int q = 0; q < G::RPT; ++q) {
        const uint32_t d = rk[q] & 0xffff;
        const uint32_t pos = base[d] + (rk[q] >> 16);
        const uint32_t slot = d * C::AREA + pos;
        const bool ok = pos < OCAP;
        const uint32_t g = g0 + (q / C::IPH) * NTG + tid;
        const uint32_t li = g * C::IPH + (q % C::IPH); // leaf index
        row_store<W0>(rs, ok ? slot * (SW0 * 4) : OOB, rw[q]);
        __builtin_amdgcn_raw_buffer_store_b32(li, rl, ok ? slot * 4 : OOB, 0, 0);
    }
    }
}

// ------------------------------------------------------------------ stages 1..K
// Parent triple of a stage-s row (s >= 1): (producing bucket << 32) | (j << 16) | i; its parents
// are the stage-(s-1) slots bucket*AREA + i and bucket*AREA + j.
__device__ __forceinline__ uint64_t pack_tri(uint32_t d, uint32_t i, uint32_t j) {
    return ((uint64_t)d << 32) | (j << 16) | i;
}
// Compact parent word (EhCfg::cp): i | j << 16, the spare high bits of each half holding d's bits
// 0..DH-1 and DH..DX-1; d's bits DX.. ride in the low bits of the row's last word.
template <class C> __host__ __device__ __forceinline__ uint32_t cpack(uint32_t d, uint32_t i, uint32_t j) {
    return i | (j << 16) | ((d & C::DHM) << C::IB) | (((d >> C::DH) & C::DHM) << (16 + C::IB));
}
template <class C> __host__ __device__ __forceinline__ uint32_t cunpack_d(uint32_t pw, uint32_t lastword) {
    return ((pw >> C::IB) & C::DHM) | (((pw >> (16 + C::IB)) & C::DHM) << C::DH) | ((lastword & C::RMASK) << C::DX);
}

// Diagnostic builds (STAMP) record s_memtime at each phase boundary (thread 0, after the
// barrier) into `stamps` — never used by the production instantiation.
#define EH_STAMP(k)                                                                                  \
    do {                                                                                             \
        if constexpr (STAMP) {                                                                       \
            if (threadIdx.x == 0) stamps[(size_t)bk * 16 + (k)] = __builtin_amdgcn_s_memtime();        \
        }                                                                                            \
    } while (0)

// LDS bytes of a round. Phase-D union `un` (bytes): {sidx[CAP] u16, bend[NRESTS] u32, then the
// pair list plist[MP*NT] u32} during the collision search; the slot -> pair table spair[MP*NT]
// u32 (aliasing plist) after it.
template <class C> constexpr int un_walk_bend(int cap) { return (cap * 2 + 3) / 4 * 4; }
template <class C> constexpr int un_walk_list(int cap) { return un_walk_bend<C>(cap) + C::NRESTS * 4; }
// Pairs per lane: one lane per LDS row slot, plus the configuration's MPX, plus BCP_EH_MP_LATE
// extra from round BCP_EH_MP_LATE_FROM on ((200,9) only): without depth-1 pruning the late rounds'
// pair lists grow past the row count (duplicate subtrees) and overflowed in round 8.
template <class C> constexpr int round_mp(int stage) {
    return stage == C::K ? 1
                         : (C::AREA_NF + C::NT - 1) / C::NT + C::MPX +
                               (C::K == 9 && stage >= BCP_EH_MP_LATE_FROM ? BCP_EH_MP_LATE : 0);
}
template <class C> constexpr int round_un(int stage) {
    const int cap = C::cap(stage);
    if (stage == C::K) return un_walk_list<C>(cap); // final round: sidx and bend only
    const int walk = un_walk_list<C>(cap) + round_mp<C>(stage) * C::NT * 4; // + the pair list
    const int pairs = round_mp<C>(stage) * C::NT * 4; // spair: every pair a lane may hold
    return walk > pairs ? walk : pairs;
}
template <class C> constexpr int round_lds(int stage, bool prune) {
    const int WR = C::words(stage - 1);
    const int WI = WR; // LDS words per row
    const int cap = C::cap(stage);
    const int pruneb = prune ? cap * 4 + (C::cp(stage - 1) ? 0 : (cap * 2 + 3) / 4 * 4) : 0;
    const int hists = stage == C::K ? 12 : 2 * C::HW * 4 + (C::NB * (C::H16 ? 2 : 4) + 3) / 4 * 4;
    return (cap * WI + 3) / 4 * 16 + pruneb + 4 + round_un<C>(stage) + hists + (C::NW + 1) * 4;
}
// Depth-1 duplicate pruning wherever its parent words fit next to the full rows.
template <class C> constexpr bool round_prunes(int stage) {
    // (the pruning start was measured on (200,9); the small configurations keep pruning from round 2)
    constexpr int from = C::K == 9 ? BCP_EH_PRUNE_FROM : 2;
    return (stage >= from || stage == C::K) && stage >= 2 && round_lds<C>(stage, true) <= C::LDS_BUDGET;
}

// STAGE < K: collision round producing stage-STAGE rows. STAGE == K: final round.
// Bucket bk = nonce*NB + d holds the stage STAGE-1 rows whose top digit bits are d (area d of
// that stage, CTRin[bk] rows).
//
// The kernel is PERSISTENT and software-pipelined: one workgroup per CU walks buckets
// blockIdx.x, +gridDim.x, ... While it collides bucket b out of LDS, the rows of its next
// bucket are in flight into VGPRs (lane-flat row loads of the contiguous area, issued in slices
// across the phases; plain loads are not drained by a bare barrier). Per bucket:
//   A. commit: prefetched rows (VGPRs) -> LDS rows (+ parent words when pruning), counting each
//      row's RB-bit key with a returning LDS atomic (its rank in the key group);
//      issue the first slice of the next bucket's loads;
//   D1. key scan: every committed row learns its sorted position;
//   D2. pair list by per-wave compaction (one barrier), then the pair filter (identical
//       subtrees; depth-1 pruning where the round prunes) and the destination histogram;
//   D3. one atomicAdd per destination bucket claims this bucket's runs there; counting sort of
//       the pairs by destination;
//   D4. one-lane-per-row emit (XOR, shift one digit, 16-byte stores) into the claimed runs,
//       plus the parent word(s).
// The final round (STAGE == K) sorts its one-word rows by key and lists the candidates: pairs
// equal on all remaining bits.
// Input rows whose slots carry compact parents keep the parent-bucket bits in their padding in
// LDS (the prune check reads them); every comparison and the emit XOR mask them out (RMI).
// pdrop[STAGE]: pairs lost to a full pair list or to the 14-partner cap of a row in a large key
// group (duplicate subtrees); pdrop[K + STAGE]: stage-(STAGE-1) rows past the
// round's capacity (offered to a bucket but never read), counted for every nonce.
template <class C, int STAGE, bool STAMP>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu(C::WGCU * C::NT / 256)))
void eh_round(const uint32_t* __restrict__ Rin, const uint32_t* __restrict__ CTRin, uint32_t* __restrict__ Rout,
              uint32_t* __restrict__ CTRout, uint32_t* __restrict__ ncand, uint64_t* __restrict__ cand,
              uint64_t* __restrict__ stamps, uint32_t* __restrict__ pdrop, int nbk) {
    constexpr int WI = C::words(STAGE - 1);
    constexpr int WO = (STAGE < C::K) ? C::words(STAGE) : 1;
    constexpr int CAP = C::cap(STAGE);                        // LDS rows / pair-list entries
    constexpr bool FINAL = STAGE == C::K;
    constexpr bool PRUNE = round_prunes<C>(STAGE);
    static_assert(round_lds<C>(STAGE, PRUNE) <= 160 * 1024 / C::WGCU, "round LDS budget");
    constexpr int NT = C::NT;
    constexpr int RPL = (CAP + NT - 1) / NT;                // prefetched rows per lane
    constexpr int MP = round_mp<C>(STAGE);                  // pairs per lane (registers)
    constexpr int SWI = C::sw(STAGE - 1);                  // words per input slot
    constexpr int SWO = STAGE < C::K ? C::sw(STAGE) : 1;   // words per output slot
    constexpr bool CPI = C::cp(STAGE - 1);                 // input slots carry one compact parent word
    constexpr uint32_t RMI = C::rmask(STAGE - 1);          // parent bits in the input rows' padding
    constexpr int SLI = (RPL + BCP_EH_PF_SLICES - 1) / BCP_EH_PF_SLICES; // prefetch slice (rows per phase)
    constexpr int BPT = (C::NB + NT - 1) / NT;             // destination buckets per thread (claims)
    // key counting folded into the commit (collision rounds): bend holds counts after the commit
    // and group starts after the scan; spair then aliases the pair list, so bend survives the
    // emit and is cleared for the next bucket in D3
    constexpr bool FOLD = !FINAL;
    using HT = std::conditional_t<C::H16, uint16_t, uint32_t>;
    __shared__ __attribute__((aligned(16))) uint32_t rows[(CAP * WI + 3) / 4 * 4];
    __shared__ uint32_t psig[PRUNE ? CAP : 1];                // the input rows' parent word (j << 16 | i, + d bits)
    __shared__ uint16_t pdw[PRUNE && !CPI ? CAP : 1];         // two-word parents: the producing bucket
    __shared__ uint32_t npairs;                                // wave-compaction pair list fill
    __shared__ __attribute__((aligned(16))) uint8_t un[round_un<C>(STAGE)];
    __shared__ uint32_t hist_[FINAL ? 1 : C::HW], cur_[FINAL ? 1 : C::HW]; // H16: two 16-bit counters per word
    __shared__ HT base[FINAL ? 1 : C::NB];
    __shared__ uint32_t wsum[C::NW + 1];
    uint16_t* sidx = reinterpret_cast<uint16_t*>(un);
    uint32_t* bend = reinterpret_cast<uint32_t*>(un + un_walk_bend<C>(CAP));
    uint32_t* plist = reinterpret_cast<uint32_t*>(un + un_walk_list<C>(CAP));
    uint32_t* spair = FOLD ? plist : reinterpret_cast<uint32_t*>(un);
    const int tid = threadIdx.x;
    const int G = gridDim.x;
    int it = 0;
    int bk = xcd_bucket<C::NB>(blockIdx.x, 0, G, nbk);
    if (bk < 0) return; // uniform per workgroup

    // histogram entry b (count or running position) and its returning increment
    auto hget = [&](const uint32_t* h, int b) -> uint32_t {
        if constexpr (C::H16) return reinterpret_cast<const uint16_t*>(h)[b];
        else return h[b];
    };
    auto hinc = [&](uint32_t* h, uint32_t b) -> uint32_t {
        if constexpr (C::H16) {
            const uint32_t sh = (b & 1) * 16;
            return (atomicAdd(&h[b >> 1], 1u << sh) >> sh) & 0xffffu;
        } else {
            return atomicAdd(&h[b], 1u);
        }
    };
    // rows i and j share a parent (depth-1 duplicate): equal producing bucket and a common LDS row
    auto shares_parent = [&](uint32_t i, uint32_t j) -> bool {
        const uint32_t a = psig[i], b = psig[j];
        const uint32_t ai = a & C::IMASK, bi = b & C::IMASK;
        const bool hit = (ai & 0xffff) == (bi & 0xffff) || (ai & 0xffff) == (bi >> 16) ||
                         (ai >> 16) == (bi & 0xffff) || (ai >> 16) == (bi >> 16);
        if (!hit) return false;
        if constexpr (CPI)
            return ((a ^ b) & ~C::IMASK) == 0 && ((rows[i * WI + WI - 1] ^ rows[j * WI + WI - 1]) & RMI) == 0;
        else
            return pdw[i] == pdw[j];
    };

    // a collision pair (LDS rows i, j) is kept unless the rows are identical or share a parent;
    // dest = its destination bucket
    auto pair_keep = [&](uint32_t i, uint32_t j, uint32_t& dest) -> bool {
        uint32_t x0 = rows[i * WI] ^ rows[j * WI];
        if constexpr (WI == 1) x0 &= ~RMI;
        // identical subtrees are dropped; word 0 differs in all but ~2^-21 of the pairs, so the
        // remaining words are read only when it matches
        bool keep = x0 != 0;
        if (!keep) {
#pragma unroll
            for (int w = 1; w < WI; ++w) {
                uint32_t y = rows[i * WI + w] ^ rows[j * WI + w];
                if (w == WI - 1) y &= ~RMI;
                keep |= y != 0;
            }
        }
        if constexpr (PRUNE) {
            if (keep && shares_parent(i, j)) keep = false;
        }
        dest = (x0 >> (32 - C::DB)) & (C::NB - 1);
        return keep;
    };

    // A thread id the compiler cannot see through: keeps the per-lane index math of the
    // prefetch/commit loops from being hoisted out of the persistent loop (live invariants
    // would otherwise push the prefetched rows out to scratch).
    auto opaque_tid = [&]() -> uint32_t {
        uint32_t t;
        asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(tid));
        return t;
    };
    // (a round that does not prune loads only the row words of each slot)
    constexpr int LWI = PRUNE ? (CPI ? WI + 1 : WI + 2) : WI;
    uint32_t nr[RPL][LWI];
    uint32_t krank[FOLD ? RPL : 1]; // FOLD: (key << 16) | rank in the key group of each committed row
    int pf_bk = bk;
    uint32_t pf_n = 0;
    // Issue prefetch rows [u0, u1) of bucket pf_bk. Every vector-memory instruction of the loop
    // body is issued unconditionally (lanes with nothing to move use an out-of-range buffer offset,
    // which the descriptor's range check drops), so the compiler can count the outstanding
    // operations and wait for the prefetched words with a precise vmcnt(N) instead of vmcnt(0): a
    // vmcnt(0) at the commit would wait for the acks of the previous bucket's emit stores as well.
    auto issue = [&](int u0, int u1) {
        const int nonce = pf_bk / C::NB, d = pf_bk % C::NB;
        const auto rs = buf_rsrc(Rin + ((size_t)nonce * C::ROWS + (size_t)d * C::AREA) * SWI, CAP * SWI * 4);
        const uint32_t ot = opaque_tid();
#pragma unroll
        for (int u = 0; u < RPL; ++u) {
            if (u < u0 || u >= u1) continue;
            const uint32_t r = ot + u * NT;
            row_load<LWI>(rs, r < pf_n ? r * (SWI * 4) : OOB, nr[u]);
        }
    };

    // prologue: first bucket in flight, fill of the second known
    uint32_t fill = CTRin[bk]; // rows offered to the current bucket (more than CAP: the rest were dropped)
    uint32_t n = min(fill, (uint32_t)CAP);
    pf_n = n;
    issue(0, RPL);
    if constexpr (!FINAL) {
        // As many (dropped) stores as one emit issues: the compiler's wait counts at the loop head
        // take the minimum over the entry and back edges; with these, both edges see the prefetch
        // loads followed by MP emit store groups, so the commit waits for its loads only.
        const auto rs_out = buf_rsrc(Rout, 0);
        const uint32_t z[SWO] = {};
#pragma unroll
        for (int u = 0; u < MP; ++u) row_store<SWO>(rs_out, OOB + 256 * u, z); // distinct offsets: identical stores would be merged
    }
    if constexpr (FOLD) {
        for (int k = tid; k < C::NRESTS; k += NT) bend[k] = 0;
        __syncthreads();
    }
    const int bk1 = xcd_bucket<C::NB>(blockIdx.x, 1, G, nbk);
    uint32_t fill_next = bk1 >= 0 ? CTRin[bk1] : 0u;
    // Fill of bucket b (0 for b < 0). As a buffer load it is counted by vmcnt, which barriers do not
    // drain; a plain load of this uniform address would be a scalar load, counted with the LDS
    // operations in lgkmcnt, and the lgkmcnt(0) before the next barrier would wait for its
    // global-memory round trip. It is read (readfirstlane) one bucket later, after the commit has
    // waited for the prefetched rows that were issued around it.
    const auto ctr_rs = buf_rsrc(CTRin, (uint32_t)nbk * 4);
    auto fill_of = [&](int b) -> uint32_t {
        return __builtin_amdgcn_raw_buffer_load_b32(ctr_rs, b >= 0 ? (uint32_t)b * 4 : OOB, 0, 0);
    };

    for (;;) {
        const int nonce = bk / C::NB, d = bk % C::NB;
        EH_STAMP(0);
        if (tid == 0 && fill > (uint32_t)CAP) atomicAdd(&pdrop[C::K + STAGE], fill - CAP); // rare
        // A. commit the prefetched bucket (one row per lane per unit)
        {
            const uint32_t ot = opaque_tid();
#pragma unroll
            for (int u = 0; u < RPL; ++u) {
                const uint32_t r = ot + u * NT;
                if (r < n) {
                    if constexpr (WI % 2 == 0) {
#pragma unroll
                        for (int w = 0; w < WI; w += 2)
                            *reinterpret_cast<u2v*>(&rows[r * WI + w]) = u2v{nr[u][w], nr[u][w + 1]};
                    } else {
#pragma unroll
                        for (int w = 0; w < WI; ++w) rows[r * WI + w] = nr[u][w];
                    }
                    if constexpr (PRUNE) {
                        psig[r] = nr[u][WI];
                        if constexpr (!CPI) pdw[r] = (uint16_t)nr[u][WI + 1];
                    }
                    if constexpr (FOLD) {
                        const uint32_t key = nr[u][0] >> (32 - C::RB);
                        krank[u] = (key << 16) | atomicAdd(&bend[key], 1u);
                    }
                }
            }
        }
        if constexpr (!FINAL)
            for (int b = tid; b < C::HW; b += NT) hist_[b] = 0;
        if constexpr (!FOLD)
            for (int k = tid; k < C::NRESTS; k += NT) bend[k] = 0;
        if (tid == 0) npairs = 0;
        EH_STAMP(1);
        const int bn = xcd_bucket<C::NB>(blockIdx.x, it + 1, G, nbk);
        const bool more = bn >= 0; // uniform
        const uint32_t fn = more ? (uint32_t)__builtin_amdgcn_readfirstlane(fill_next) : 0u;
        const uint32_t nn = min(fn, (uint32_t)CAP);
        pf_bk = more ? bn : bk;
        pf_n = nn;
        const int bn2 = xcd_bucket<C::NB>(blockIdx.x, it + 2, G, nbk);
        issue(0, SLI); // nothing moves when !more (pf_n = 0), but the instruction count stays fixed
        fill_next = fill_of(bn2);
        __syncthreads();
        EH_STAMP(2);

        // D1. key sort. FOLD: the commit counted the keys; scan to group starts and place each
        //     row by its rank: sorted position (krank, reused) and the number of later positions
        //     in the row's key group (its pairs, capped at 14 as below). Final round: count,
        //     scan, then place (sidx = row ids grouped by key, bend[key] = end of the key's group).
        auto key_of = [&](uint32_t i) -> uint32_t { return rows[i * WI] >> (32 - C::RB); };
        uint32_t kpairs[FOLD ? RPL : 1];
        if constexpr (FOLD) {
            block_exscan<NT, (C::NRESTS + NT - 1) / NT>(bend, C::NRESTS, wsum);
            const uint32_t ot = opaque_tid();
#pragma unroll
            for (int u = 0; u < RPL; ++u) {
                const uint32_t r = ot + u * NT;
                kpairs[u] = 0;
                if (r < n) {
                    const uint32_t key = krank[u] >> 16;
                    const uint32_t pos = bend[key] + (krank[u] & 0xffff);
                    const uint32_t e = key + 1 < (uint32_t)C::NRESTS ? bend[key + 1] : n;
                    sidx[pos] = (uint16_t)r;
                    krank[u] = pos;
                    kpairs[u] = min(e - pos - 1, 14u);
                    if (e - pos - 1 > 14u) atomicAdd(&pdrop[STAGE], e - pos - 1 - 14u); // capped pairs (rare) count as pair-list drops
                }
            }
        } else {
            for (uint32_t i = tid; i < n; i += NT) atomicAdd(&bend[key_of(i)], 1u);
            __syncthreads();
            block_exscan<NT, (C::NRESTS + NT - 1) / NT>(bend, C::NRESTS, wsum);
            for (uint32_t i = tid; i < n; i += NT) sidx[atomicAdd(&bend[key_of(i)], 1u)] = (uint16_t)i;
        }
        issue(SLI, 2 * SLI);
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
                    if ((rows[j] ^ ri) & ~RMI) continue;
                    if constexpr (PRUNE) {
                        if (shares_parent(i, j)) continue;
                    }
                    const uint32_t c = atomicAdd(&ncand[nonce], 1u);
                    if (c < (uint32_t)C::MAXCAND) cand[(size_t)nonce * C::MAXCAND + c] = pack_tri(d, i, j);
                }
            }
            issue(2 * SLI, RPL);
        } else {
            // D2. pair list by per-wave compaction. Sorted position p pairs with every later
            //     position of its key group: c_p = bend[key] - p - 1 pairs (capped at 14; a group
            //     of 16+ rows is ~1e-8 likely). Each lane counts the pairs of the rows it
            //     committed (from registers), a DPP wave scan gives the lane's offset inside its
            //     wave, ONE LDS atomic per wave claims the wave's block of the list, and the lane
            //     writes its (j << 16 | i) pairs there: one barrier. The list holds MP*NT pairs
            //     (above the row capacity: capped pair lists lost ~9% of the solutions); identical
            //     subtrees and pairs that share a parent are dropped when the pairs are read back.
            uint32_t cnt = 0;
#pragma unroll
            for (int u = 0; u < RPL; ++u) cnt += kpairs[u];
            const uint32_t incl = wave_incl<false>(cnt);
            uint32_t wb = 0;
            if ((tid & 63) == 63) wb = atomicAdd(&npairs, incl);
            uint32_t o = __builtin_amdgcn_readlane(wb, 63) + incl - cnt;
#pragma unroll
            for (int u = 0; u < RPL; ++u) {
                if (!kpairs[u]) continue;
                const uint32_t p = krank[u];
                const uint32_t i = tid + u * NT;
                for (uint32_t q = p + 1; q <= p + kpairs[u]; ++q, ++o) {
                    if (o >= (uint32_t)(MP * NT)) continue;
                    plist[o] = ((uint32_t)sidx[q] << 16) | i;
                }
            }
            __syncthreads();
            EH_STAMP(7); // pair list complete (splits D2 into listing and filtering)
            const uint32_t P = npairs;
            const uint32_t Pc = min(P, (uint32_t)(MP * NT));
            if (tid == 0 && P > (uint32_t)(MP * NT)) atomicAdd(&pdrop[STAGE], P - MP * NT); // rare
            uint32_t pv[MP], pd[MP];
#pragma unroll
            for (int u = 0; u < MP; ++u) {
                const uint32_t k = tid + u * NT;
                pv[u] = NIL;
                pd[u] = 0;
                if (k < Pc) {
                    const uint32_t pr = plist[k];
                    const uint32_t i = pr & 0xffff, j = pr >> 16;
                    uint32_t dest;
                    if (pair_keep(i, j, dest)) {
                        pv[u] = (j << 16) | i;
                        pd[u] = dest; // destination bucket
                        hinc(hist_, pd[u]);
                    }
                }
            }
            // bend's last reads were before the barrier above; the next commit counts here
            for (int k = tid; k < C::NRESTS; k += NT) bend[k] = 0;
            __syncthreads();
            EH_STAMP(4);
            // D3. claim this bucket's runs in the destination areas (device-scope atomics whose
            //     latency hides behind the scan and the scatter), then sort the pairs by
            //     destination: each pair takes the next LDS slot of its destination's run.
            //     Thread t owns destinations [t*BPT, t*BPT + BPT) (the scan's entry split).
            uint32_t myb[BPT];
#pragma unroll
            for (int k = 0; k < BPT; ++k) {
                const int b = tid * BPT + k;
                myb[k] = 0;
                if (b < C::NB) myb[k] = atomicAdd(&CTRout[(size_t)nonce * C::NB + b], hget(hist_, b)); // wave-uniform branch
            }
            issue(2 * SLI, RPL); // after the claim: waiting for its return then skips these loads
            uint32_t start = 0; // first LDS slot of the thread's first destination
            uint32_t np;
            if constexpr (C::H16)
                np = block_exscan<NT, BPT, uint16_t, uint16_t>(reinterpret_cast<const uint16_t*>(hist_),
                                                               reinterpret_cast<uint16_t*>(cur_), C::NB, wsum, &start);
            else
                np = block_exscan<NT, BPT>(hist_, cur_, C::NB, wsum, &start);
#pragma unroll
            for (int u = 0; u < MP; ++u)
                if (pv[u] != NIL) spair[hinc(cur_, pd[u])] = pv[u];
#pragma unroll
            for (int k = 0; k < BPT; ++k) { // LDS slot t of destination b -> run position base[b] + t
                const int b = tid * BPT + k;
                if (b < C::NB) {
                    base[b] = (HT)(myb[k] - start);
                    start += hget(hist_, b);
                }
            }
            __syncthreads();
            EH_STAMP(5);
            // D4. emit, one lane per output row in destination order: XOR, shift one digit,
            //     store into the claimed run (rows past the next round's capacity are dropped)
            constexpr uint32_t OCAP = C::cap(STAGE + 1 <= C::K ? STAGE + 1 : C::K);
            constexpr uint32_t RMO = C::rmask(STAGE);
            const auto rs_out = buf_rsrc(Rout + (size_t)nonce * C::ROWS * SWO, (uint32_t)(C::ROWS * SWO * 4));
#pragma unroll
            for (int u = 0; u < MP; ++u) { // fixed trip count, unconditional stores (see issue())
                const uint32_t t = tid + u * NT;
                const uint32_t pr = t < np ? spair[t] : 0u;
                const uint32_t i = pr & 0xffff, j = pr >> 16; // LDS rows = the parents' slots in the input area
                uint32_t x[WI + 1], o[WO];
                lds_row_xor<WI>(rows, i, j, x);
                x[WI - 1] &= ~RMI;
                x[WI] = 0;
                const uint32_t b = (x[0] >> (32 - C::DB)) & (C::NB - 1);
                const uint32_t pos = (HT)(base[b] + t);
                const bool ok = t < np && pos < OCAP;
                const uint32_t slot = b * C::AREA + pos;
#pragma unroll
                for (int w = 0; w < WO; ++w) o[w] = (x[w] << C::DB) | (x[w + 1] >> (32 - C::DB));
                uint32_t ov[SWO] = {};
#pragma unroll
                for (int w = 0; w < WO; ++w) ov[w] = o[w];
                if constexpr (C::cp(STAGE)) {
                    ov[WO - 1] |= (d >> C::DX) & RMO;
                    ov[WO] = cpack<C>(d, i, j);
                } else {
                    ov[WO] = (j << 16) | i;
                    ov[WO + 1] = d;
                }
                row_store<SWO>(rs_out, ok ? slot * (SWO * 4) : OOB, ov);
            }
        }
        __syncthreads();
        EH_STAMP(6);
        if (!more) break;
        bk = bn;
        ++it;
        fill = fn;
        n = nn;
    }
}


// ------------------------------------------------------------------ tree expansion
// The stage arrays (stage-s slot = row, parent word(s)) passed by value; LEAF: stage-0 leaf
// index per slot.
struct EhStages {
    const uint32_t* r[16];
};
template <class C>
__global__ __launch_bounds__(C::L < 64 ? 64 : C::L) void eh_expand(const uint32_t* __restrict__ LEAF, EhStages st,
                                                                  const uint32_t* __restrict__ ncand,
                                                                  const uint64_t* __restrict__ cand,
                                                                  uint32_t* __restrict__ out_idx,
                                                                  uint32_t* __restrict__ out_valid,
                                                                  uint32_t* __restrict__ nout,
                                                                  uint32_t* __restrict__ out_list) {
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
    // level s: 2^(K-s) triples of round s -> 2^(K-s+1) stage-(s-1) slots -> their triples. A
    // parent outside the slot arrays (never produced by a correct round) is clamped to slot 0
    // and the candidate is rejected, so no corrupt word can address past the stage arrays.
    for (int s = C::K; s >= 1; --s) {
        __syncthreads();
        const uint32_t cnt = 1u << (C::K - s);
        if (t < 2 * cnt) {
            const uint64_t tr = tri[t >> 1];
            const uint32_t dd = (uint32_t)(tr >> 32);
            const uint32_t r = (t & 1) ? (((uint32_t)tr >> 16) & 0xffff) : ((uint32_t)tr & 0xffff);
            const bool in = dd < (uint32_t)C::NB && r < (uint32_t)C::AREA;
            if (!in) dup = 1;
            buf[cur][t] = in ? dd * C::AREA + r : 0u;
        }
        __syncthreads();
        if (s > 1 && t < 2 * cnt) { // stage s-1 slot: row words, then the parent word(s)
            const uint32_t* q = st.r[s - 1] + ((size_t)nonce * C::ROWS + buf[cur][t]) * C::sw(s - 1) + C::words(s - 1);
            if (C::cp(s - 1))
                tri[t] = ((uint64_t)cunpack_d<C>(q[0], q[-1]) << 32) | (q[0] & C::IMASK);
            else
                tri[t] = ((uint64_t)q[1] << 32) | q[0];
        }
    }
    __syncthreads();
    if (t < (uint32_t)L) buf[cur][t] = LEAF[(size_t)nonce * C::ROWS + buf[cur][t]];
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
    // Valid solutions are also appended to one compact list, (nonce, candidate, L indices) per
    // entry, so the host copies a few KB per nonce instead of MAXCAND * L words.
    if (dup) return; // uniform
    __shared__ uint32_t slot;
    if (t == 0) slot = atomicAdd(nout, 1u);
    __syncthreads();
    uint32_t* e = out_list + (size_t)slot * (L + 2);
    if (t == 0) {
        e[0] = nonce;
        e[1] = c;
    }
    if (t < (uint32_t)L) e[2 + t] = buf[cur][t];
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
    hipEvent_t ev_gen = nullptr, ev_rounds = nullptr; // this solver's last generation / rounds done (pipelining)
    const Impl* after = nullptr;                        // Launch(states, prev): the batch to pipeline behind
    DevBuf<bcpk::EhBaseState> d_states;
    DevBuf<uint32_t> d_ctr, d_leaf, d_ncand, d_idx, d_valid, d_pdrop, d_nout, d_out;
    DevBuf<uint64_t> d_cand;
    DevBuf<uint32_t> d_rst[16]; // merged layout: stage-s slot arrays (s = 0..K-1)
    HostBuf<bcpk::EhBaseState> h_states;
    HostBuf<uint32_t> h_ncand, h_idx, h_ctr0, h_ctr_all, h_pdrop, h_nout, h_out;
    size_t outq = 0; // compact-list entries copied back with every batch (more: a second copy)
    size_t rows = 0, L = 0, maxcand = 0, nb = 0, kstages = 0;
    std::vector<size_t> caps; // caps[s]: LDS capacity of the round that reads stage-s rows
    std::vector<size_t> slot_words, row_words; // per stage
    uint32_t cp_ib = 0, cp_dh = 0, cp_dhm = 0, cp_dx = 0, cp_rmask = 0, cp_imask = 0; // compact parent layout
    std::vector<bool> compact;                  // per stage: compact parent word
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
        slot_words.clear();
        compact.clear();
        row_words.clear();
        for (int st = 0; st < C::K; ++st) {
            slot_words.push_back(C::sw(st));
            compact.push_back(C::cp(st));
            row_words.push_back(C::words(st));
        }
        kstages = C::K;
        d_states.alloc(batch);
        h_states.alloc(batch);
        static_assert(C::K <= 16, "stage arrays");
        for (int s = 0; s < C::K; ++s) d_rst[s].alloc((size_t)batch * C::ROWS * C::sw(s));
        d_ctr.alloc((size_t)C::K * batch * C::NB);
        d_leaf.alloc((size_t)batch * C::ROWS);
        cp_ib = C::IB, cp_dh = C::DH, cp_dhm = C::DHM, cp_dx = C::DX, cp_rmask = C::RMASK, cp_imask = C::IMASK;
        d_ncand.alloc(batch);
        d_pdrop.alloc(2 * C::K + 2); // [1..K]: pair-list drops per round, [K+1..2K]: row drops per stage
        h_pdrop.alloc(2 * C::K + 2);
        d_cand.alloc((size_t)batch * C::MAXCAND);
        d_idx.alloc((size_t)batch * C::MAXCAND * C::L);
        d_valid.alloc((size_t)batch * C::MAXCAND);
        h_ncand.alloc(batch);
        d_nout.alloc(1);
        h_nout.alloc(1);
        d_out.alloc((size_t)batch * C::MAXCAND * (C::L + 2));
        h_out.alloc((size_t)batch * C::MAXCAND * (C::L + 2));
        outq = std::min<size_t>((size_t)batch * 4 + 16, (size_t)batch * C::MAXCAND);
        h_idx.alloc((size_t)C::MAXCAND * C::L);
        h_ctr0.alloc((size_t)C::K * C::NB);
        h_ctr_all.alloc((size_t)C::K * batch * C::NB);
        d_stamps.alloc((size_t)C::K * batch * C::NB * 16);
        bytes = d_leaf.n * 4 + d_ctr.n * 4 + d_idx.n * 4;
        for (int s = 0; s < C::K; ++s) bytes += d_rst[s].n * 4;
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
        const uint32_t* rin = d_rst[S - 1].p;
        uint32_t* rout = S < C::K ? d_rst[S].p : nullptr;
        const uint32_t* cin = d_ctr.p + (size_t)(S - 1) * batch * C::NB;
        uint32_t* cout = S < C::K ? d_ctr.p + (size_t)S * batch * C::NB : nullptr;
        const int nbk = C::NB * nstates;
        if (stamp_mode) {
            uint64_t* st = d_stamps.p + (size_t)(S - 1) * batch * C::NB * 16;
            hipLaunchKernelGGL((bcpk::eh_round<C, S, true>), dim3(round_grid<C, S, true>(nbk)), dim3(C::NT), 0,
                               stream, rin, cin, rout, cout, d_ncand.p, d_cand.p, st, d_pdrop.p, nbk);
        } else {
            hipLaunchKernelGGL((bcpk::eh_round<C, S, false>), dim3(round_grid<C, S, false>(nbk)), dim3(C::NT), 0,
                               stream, rin, cin, rout, cout, d_ncand.p, d_cand.p, nullptr, d_pdrop.p, nbk);
        }
    }
    template <class C, int... S> void launch_rounds(int nstates, std::integer_sequence<int, S...>) {
        (launch_round<C, S + 1>(nstates), ...);
    }

    template <class C> void launch(size_t nstates) {
        BCP_HIP_CHECK(hipMemcpyAsync(d_states.p, h_states.p, nstates * sizeof(bcpk::EhBaseState),
                                     hipMemcpyHostToDevice, stream));
        BCP_HIP_CHECK(hipMemsetAsync(d_ncand.p, 0, batch * sizeof(uint32_t), stream));
        BCP_HIP_CHECK(hipMemsetAsync(d_nout.p, 0, sizeof(uint32_t), stream));
        BCP_HIP_CHECK(hipMemsetAsync(d_pdrop.p, 0, d_pdrop.n * sizeof(uint32_t), stream));
        BCP_HIP_CHECK(hipMemsetAsync(d_ctr.p, 0, d_ctr.n * sizeof(uint32_t), stream));
        if (debug) {
            if (d_leaf.n) BCP_HIP_CHECK(hipMemsetAsync(d_leaf.p, 0xff, d_leaf.n * sizeof(uint32_t), stream));
            for (int s = 0; s < C::K; ++s)
                if (d_rst[s].n) BCP_HIP_CHECK(hipMemsetAsync(d_rst[s].p, 0xff, d_rst[s].n * sizeof(uint32_t), stream));
        }
        BCP_HIP_CHECK(hipEventRecord(ev0, stream));
        // header-shaped inputs (140 B: g lands at byte 12 of the final block) take the
        // zero-message-word BLAKE2b specialisation
        bool hdr = true;
        for (size_t i = 0; i < nstates; ++i) {
            const bcpk::EhBaseState& st = h_states.p[i];
            hdr &= st.g_byte == 12;
            for (int w = 2; w < 16; ++w) hdr &= st.m[w] == 0;
        }
        uint32_t* r0 = d_rst[0].p;
        hipStream_t gs = stream;
        if (after) BCP_HIP_CHECK(hipStreamWaitEvent(gs, after->ev_gen, 0)); // one generation at a time
        constexpr bool reg = bcpk::GenReg<C, C::GNT, C::GHPT>::OK;
        if constexpr (reg) {
            using GR = bcpk::GenReg<C, C::GNT, C::GHPT>;
            const int items = GR::GWG * (int)nstates;
            const int grid = items;
            if (hdr)
                hipLaunchKernelGGL((bcpk::eh_gen_reg<C, true, C::GNT, C::GHPT>), dim3(grid), dim3(C::GNT), 0, gs,
                                   d_states.p, r0, d_leaf.p, d_ctr.p, items);
            else
                hipLaunchKernelGGL((bcpk::eh_gen_reg<C, false, C::GNT, C::GHPT>), dim3(grid), dim3(C::GNT), 0, gs,
                                   d_states.p, r0, d_leaf.p, d_ctr.p, items);
        } else if (hdr)
            hipLaunchKernelGGL((bcpk::eh_gen<C, true>), dim3(C::GENWG * nstates), dim3(C::NTG), 0, gs,
                               d_states.p, r0, d_leaf.p, d_ctr.p);
        else
            hipLaunchKernelGGL((bcpk::eh_gen<C, false>), dim3(C::GENWG * nstates), dim3(C::NTG), 0, gs,
                               d_states.p, r0, d_leaf.p, d_ctr.p);
        BCP_HIP_CHECK(hipEventRecord(ev_gen, gs));
        if (after) BCP_HIP_CHECK(hipStreamWaitEvent(stream, after->ev_rounds, 0)); // one round chain at a time
        launch_rounds<C>((int)nstates, std::make_integer_sequence<int, C::K>{});
        constexpr int EB = C::L < 64 ? 64 : C::L;
        bcpk::EhStages stages{};
        for (int s = 0; s < C::K; ++s) stages.r[s] = d_rst[s].p;
        hipLaunchKernelGGL((bcpk::eh_expand<C>), dim3(C::MAXCAND * nstates), dim3(EB), 0, stream, d_leaf.p, stages,
                           d_ncand.p, d_cand.p, d_idx.p, d_valid.p, d_nout.p, d_out.p);
        BCP_HIP_CHECK(hipEventRecord(ev_rounds, stream));
        BCP_HIP_CHECK(hipGetLastError());
        BCP_HIP_CHECK(hipEventRecord(ev1, stream));
        BCP_HIP_CHECK(
            hipMemcpyAsync(h_ncand.p, d_ncand.p, nstates * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        // pair-list and row drops of every nonce (a few words)
        BCP_HIP_CHECK(hipMemcpyAsync(h_pdrop.p, d_pdrop.p, d_pdrop.n * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        if (debug) { // per-stage fills of nonce 0's buckets
            for (int s = 0; s < C::K; ++s)
                BCP_HIP_CHECK(hipMemcpyAsync(h_ctr0.p + (size_t)s * C::NB, d_ctr.p + (size_t)s * batch * C::NB,
                                             C::NB * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
            BCP_HIP_CHECK(hipMemcpyAsync(h_ctr_all.p, d_ctr.p, d_ctr.n * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        }
        BCP_HIP_CHECK(hipMemcpyAsync(h_nout.p, d_nout.p, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        BCP_HIP_CHECK(hipMemcpyAsync(h_out.p, d_out.p, outq * (C::L + 2) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                     stream));
        if (debug) // every candidate of nonce 0, valid or not
            BCP_HIP_CHECK(hipMemcpyAsync(h_idx.p, d_idx.p, C::MAXCAND * C::L * sizeof(uint32_t),
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
    BCP_HIP_CHECK(hipEventCreateWithFlags(&impl->ev_gen, hipEventDisableTiming));
    BCP_HIP_CHECK(hipEventCreateWithFlags(&impl->ev_rounds, hipEventDisableTiming));
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
        if (impl->ev_gen) (void)hipEventDestroy(impl->ev_gen);
        if (impl->ev_rounds) (void)hipEventDestroy(impl->ev_rounds);
    }
}

unsigned EquihashGpuSolver::N() const { return impl->n; }
unsigned EquihashGpuSolver::K() const { return impl->k; }
int EquihashGpuSolver::Batch() const { return impl->batch; }
const EhGpuStats& EquihashGpuSolver::Stats() const { return impl->stats; }
void EquihashGpuSolver::SetDebug(bool on) { impl->debug = on; }
void EquihashGpuSolver::SetStampMode(bool on) { impl->stamp_mode = on; }

// Mean cycles per phase per round (diagnostic stamp builds): [stage][phase delta], deltas
// 1..6 = commit, next-bucket issue + barrier, key sort, pair enumeration, claim + pair sort, emit;
// [0] = whole bucket.
std::vector<std::vector<double>> EquihashGpuSolver::PhaseCycles(int nonces) {
    BCP_HIP_CHECK(hipSetDevice(impl->device));
    BCP_HIP_CHECK(hipStreamSynchronize(impl->stream));
    const size_t per = (size_t)impl->batch * impl->nb * 16;
    std::vector<uint64_t> h(impl->kstages * per);
    BCP_HIP_CHECK(hipMemcpy(h.data(), impl->d_stamps.p, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<std::vector<double>> out;
    for (size_t s = 0; s < impl->kstages; ++s) {
        // phases 1..6, then D2 split at stamp 7: listing (3 -> 7) and filtering (7 -> 4)
        std::vector<double> acc(9, 0.0);
        size_t cnt = 0;
        for (size_t wg = 0; wg < (size_t)nonces * impl->nb; ++wg) {
            const uint64_t* t = &h[s * per + wg * 16];
            if (t[0] == 0) continue;
            for (int k = 1; k < 7; ++k)
                if (t[k] >= t[k - 1] && t[k] != 0) acc[k] += (double)(t[k] - t[k - 1]);
            acc[0] += (double)(t[6] - t[0]);
            if (t[7] >= t[3] && t[4] >= t[7] && t[7] != 0) {
                acc[7] += (double)(t[7] - t[3]);
                acc[8] += (double)(t[4] - t[7]);
            }
            ++cnt;
        }
        for (auto& a : acc) a = cnt ? a / cnt : 0;
        out.push_back(acc);
    }
    return out;
}
void EquihashGpuSolver::ResetStats() { impl->stats = EhGpuStats(); }

// Debug: nonce 0 of the last batch, K arrays of ROWS slots: stage-0 leaf indices (zero-extended),
// then the parent triples of stages 1..K-1; with SetDebug(true) never-written slots read all-ones.
std::vector<uint64_t> EquihashGpuSolver::DebugDump() {
    BCP_HIP_CHECK(hipSetDevice(impl->device));
    BCP_HIP_CHECK(hipStreamSynchronize(impl->stream));
    const Impl& m = *impl;
    const size_t R = m.rows, K = m.kstages;
    std::vector<uint64_t> out(K * R);
    std::vector<uint32_t> leaf(R);
    BCP_HIP_CHECK(hipMemcpy(leaf.data(), m.d_leaf.p, R * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < R; ++i) out[i] = leaf[i];
    // the parent word(s) follow the row in every stage-s slot of nonce 0 (bcpk::cpack layout)
    auto cunpack_d = [&](uint32_t pw, uint32_t last) {
        return ((pw >> m.cp_ib) & m.cp_dhm) | (((pw >> (16 + m.cp_ib)) & m.cp_dhm) << m.cp_dh) |
               ((last & m.cp_rmask) << m.cp_dx);
    };
    for (size_t s = 1; s < K; ++s) {
        const size_t sw = m.slot_words[s], w = m.row_words[s];
        std::vector<uint32_t> buf(R * sw);
        BCP_HIP_CHECK(hipMemcpy(buf.data(), m.d_rst[s].p, R * sw * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < R; ++i) {
            const uint32_t* q = &buf[i * sw + w];
            if (m.compact[s] && q[0] == 0xffffffffu) // never written (SetDebug fill): no LDS row index is all-ones
                out[s * R + i] = ~0ull;
            else
                out[s * R + i] = m.compact[s] ? ((uint64_t)cunpack_d(q[0], q[-1]) << 32) | (q[0] & m.cp_imask)
                                              : ((uint64_t)q[1] << 32) | q[0];
        }
    }
    return out;
}
size_t EquihashGpuSolver::DeviceBytes() const { return impl->bytes; }

std::vector<uint32_t> EquihashGpuSolver::DebugExpandCorrupt(int mode) {
    BCP_HIP_CHECK(hipSetDevice(impl->device));
    BCP_HIP_CHECK(hipStreamSynchronize(impl->stream));
    Impl& m = *impl;
    uint32_t nc = 0;
    BCP_HIP_CHECK(hipMemcpy(&nc, m.d_ncand.p, 4, hipMemcpyDeviceToHost));
    nc = std::min<uint32_t>(nc, (uint32_t)m.maxcand);
    if (nc == 0) return {};
    uint64_t tri = 0;
    BCP_HIP_CHECK(hipMemcpy(&tri, m.d_cand.p, 8, hipMemcpyDeviceToHost));
    const size_t st = m.kstages - 1; // the stage the final round read
    const uint32_t d = (uint32_t)(tri >> 32), i = (uint32_t)tri & 0xffff;
    uint32_t* slot = m.d_rst[st].p + ((size_t)d * (m.rows / m.nb) + i) * m.slot_words[st] + m.row_words[st];
    if (mode != 0) {
        if (m.compact[st]) {
            // compact word: i | j << 16 with the bucket's bits in the spare high bits of each half
            uint32_t w = 0;
            BCP_HIP_CHECK(hipMemcpy(&w, slot, 4, hipMemcpyDeviceToHost));
            w = mode == 1 ? (w | (m.cp_dhm << m.cp_ib) | (m.cp_dhm << (16 + m.cp_ib))) : (w | ((1u << m.cp_ib) - 1));
            BCP_HIP_CHECK(hipMemcpy(slot, &w, 4, hipMemcpyHostToDevice));
        } else {
            uint32_t w[2];
            BCP_HIP_CHECK(hipMemcpy(w, slot, 8, hipMemcpyDeviceToHost));
            if (mode == 1) w[1] = 0xffffu;         // producing bucket far past NB
            else w[0] = (w[0] & 0xffff0000u) | 0xffffu; // LDS row far past the area
            BCP_HIP_CHECK(hipMemcpy(slot, w, 8, hipMemcpyHostToDevice));
        }
    }
    BCP_HIP_CHECK(hipMemsetAsync(m.d_nout.p, 0, 4, m.stream));
    dispatch_cfg(m.n, m.k, [&](auto c) {
        using C = decltype(c);
        constexpr int EB = C::L < 64 ? 64 : C::L;
        bcpk::EhStages stages{};
        for (int s2 = 0; s2 < C::K; ++s2) stages.r[s2] = m.d_rst[s2].p;
        hipLaunchKernelGGL((bcpk::eh_expand<C>), dim3(C::MAXCAND), dim3(EB), 0, m.stream, m.d_leaf.p, stages,
                           m.d_ncand.p, m.d_cand.p, m.d_idx.p, m.d_valid.p, m.d_nout.p, m.d_out.p);
    });
    BCP_HIP_CHECK(hipGetLastError());
    BCP_HIP_CHECK(hipStreamSynchronize(m.stream));
    std::vector<uint32_t> valid(nc);
    BCP_HIP_CHECK(hipMemcpy(valid.data(), m.d_valid.p, nc * 4, hipMemcpyDeviceToHost));
    return valid;
}

void EquihashGpuSolver::Launch(const std::vector<EhBaseState>& states) {
    if (states.empty() || (int)states.size() > impl->batch) throw std::invalid_argument("bad number of states");
    if (impl->inflight) throw std::runtime_error("EquihashGpuSolver: Collect() the previous launch first");
    BCP_HIP_CHECK(hipSetDevice(impl->device));
    memcpy(impl->h_states.p, states.data(), states.size() * sizeof(EhBaseState));
    dispatch_cfg(impl->n, impl->k, [&](auto c) { impl->launch<decltype(c)>(states.size()); });
    impl->inflight = (int)states.size();
}

void EquihashGpuSolver::Launch(const std::vector<EhBaseState>& states, const EquihashGpuSolver& prev) {
    if (&prev == this) throw std::invalid_argument("EquihashGpuSolver: cannot pipeline behind itself");
    if (prev.impl->device != impl->device) throw std::invalid_argument("EquihashGpuSolver: pipelined solvers on different devices");
    impl->after = prev.impl.get();
    try {
        Launch(states);
    } catch (...) {
        impl->after = nullptr;
        throw;
    }
    impl->after = nullptr;
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
    {
        // every nonce: pair-list drops per round and rows past a round's capacity per stage (accumulated)
        const size_t K = impl->kstages;
        impl->stats.pair_dropped_all.resize(K + 1, 0);
        impl->stats.stage_dropped_all.resize(K, 0);
        for (size_t r = 0; r <= K; ++r) impl->stats.pair_dropped_all[r] += impl->h_pdrop.p[r];
        for (size_t s = 0; s < K; ++s) impl->stats.stage_dropped_all[s] += impl->h_pdrop.p[K + 1 + s];
    }
    if (impl->debug) {
        // nonce 0: per stage, rows offered to each bucket (its fill counter) vs the LDS capacity
        // of the round that reads it
        const size_t NB = impl->nb;
        impl->stats.stage_rows.assign(impl->kstages, 0);
        impl->stats.stage_dropped.assign(impl->kstages, 0);
        impl->stats.stage_maxfill.assign(impl->kstages, 0);
        impl->stats.stage_top.assign(impl->kstages, {});
        impl->stats.pair_dropped.assign(impl->h_pdrop.p, impl->h_pdrop.p + impl->kstages + 1);
        // every nonce of the batch: the fullest bucket per stage and the buckets past capacity
        impl->stats.stage_maxfill_all.assign(impl->kstages, 0);
        for (size_t s = 0; s < impl->kstages; ++s)
            for (size_t x = 0; x < (size_t)ns * NB; ++x) {
                const uint64_t fill = impl->h_ctr_all.p[(s * impl->batch) * NB + x];
                impl->stats.stage_maxfill_all[s] = std::max<uint64_t>(impl->stats.stage_maxfill_all[s], fill);
                if (fill > impl->caps[s]) impl->stats.overflow_fills.push_back((uint64_t)s << 32 | fill);
            }
        for (size_t s = 0; s < impl->kstages; ++s) {
            std::vector<uint64_t> fills;
            for (size_t dd = 0; dd < NB; ++dd) {
                const uint64_t fill = impl->h_ctr0.p[s * NB + dd];
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
    const size_t ew = impl->L + 2; // compact-list entry: nonce, candidate, L indices
    const size_t nout = impl->h_nout.p[0];
    if (nout > impl->outq) // more valid solutions than the per-batch copy holds: fetch the rest
        BCP_HIP_CHECK(hipMemcpy(impl->h_out.p + impl->outq * ew, impl->d_out.p + impl->outq * ew,
                                (nout - impl->outq) * ew * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (impl->debug) {
        impl->stats.debug_cands.clear();
        const uint32_t nc = std::min<uint32_t>(impl->h_ncand.p[0], (uint32_t)impl->maxcand);
        for (uint32_t c = 0; c < nc; ++c) {
            const uint32_t* p = impl->h_idx.p + (size_t)c * impl->L;
            impl->stats.debug_cands.emplace_back(p, p + impl->L);
        }
    }
    uint64_t cands = 0;
    for (int nn = 0; nn < ns; ++nn) {
        const uint32_t c = impl->h_ncand.p[nn];
        cands += std::min<uint32_t>(c, (uint32_t)impl->maxcand);
        impl->stats.cand_max = std::max<uint64_t>(impl->stats.cand_max, c);
        if (c > impl->maxcand) impl->stats.cand_dropped += c - impl->maxcand; // lost candidates, maybe solutions
    }
    impl->stats.candidates += cands;
    impl->stats.duplicates += cands - nout;
    // the list is in completion order: put every nonce's solutions in candidate order
    std::vector<std::pair<uint64_t, const uint32_t*>> ents;
    ents.reserve(nout);
    for (size_t e = 0; e < nout; ++e) {
        const uint32_t* p = impl->h_out.p + e * ew;
        if (p[0] < (uint32_t)ns) ents.emplace_back(((uint64_t)p[0] << 32) | p[1], p + 2);
    }
    std::sort(ents.begin(), ents.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (const auto& en : ents) {
        const int nn = (int)(en.first >> 32);
        std::vector<uint32_t> v(en.second, en.second + impl->L);
        bool seen = false;
        for (auto& prev : out[nn]) seen |= (prev == v);
        if (seen) continue;
        out[nn].push_back(std::move(v));
        impl->stats.solutions++;
    }
    return out;
}

std::vector<std::vector<std::vector<uint32_t>>> EquihashGpuSolver::Solve(const std::vector<EhBaseState>& states) {
    Launch(states);
    return Collect();
}

} // namespace gpu
} // namespace bcp
