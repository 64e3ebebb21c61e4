// Equihash solver for CDNA4 (gfx950) — the GPU replacement for the reference's
// CPU BasicSolve/OptimisedSolve (reference src/crypto/equihash.cpp:332-722,
// called from generateBlocks src/rpc/mining.cpp:161-199).
//
// Algorithm (bucketed parent-pointer Wagner solver):
//   stage 0   eh_gen:    one lane per BLAKE2b call; each of the 512/N digest slices becomes a row,
//                        bucketed on the top BUCKBITS of digit 0; the rest of the bit string is stored
//                        pre-shifted so every later round reads its digit at bit 0.
//   stage 1..K-1 eh_round: one workgroup per bucket; rows are staged into LDS, chained by their
//                        RESTBITS remainder through an LDS hash table (atomicExch heads), every
//                        colliding pair is XORed, shifted by one digit and scattered to its next
//                        bucket; a 32-bit parent reference (bucket, slotA, slotB) is kept per row.
//   stage K   eh_final:  pairs colliding on the whole remaining 2 digits are solution candidates.
//   eh_expand:           one workgroup per candidate walks the K levels of parent references in
//                        LDS, canonicalises subtree order (left-first-index < right-first-index,
//                        reference IsValidSolution ordering rule) and rejects duplicate indices with
//                        an LDS bitonic sort.
// Memory (200,9): 4096 buckets x 640 slots; hash rows ping-pong between two buffers, refs are kept
// per stage (4 B/row/stage) so no index list ever grows.
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

template <int N_, int K_, int BB_, int NSLOTS_, int SB_, int MAXCAND_>
struct EhCfg {
    static constexpr int N = N_, K = K_;
    static constexpr int DB = N / (K + 1);
    static constexpr int BUCKBITS = BB_;
    static constexpr int RESTBITS = DB - BB_;
    static constexpr int NBUCKETS = 1 << BB_;
    static constexpr int NRESTS = 1 << RESTBITS;
    static constexpr int NSLOTS = NSLOTS_;
    static constexpr int SLOTBITS = SB_;
    static constexpr uint32_t SLOTMASK = (1u << SB_) - 1;
    static constexpr int INIT = 1 << (DB + 1);
    static constexpr int IPH = 512 / N;
    static constexpr int NBYTES = N / 8;
    static constexpr int NHASH = (INIT + IPH - 1) / IPH;
    static constexpr int MAXCAND = MAXCAND_;
    static constexpr int L = 1 << K;
    static constexpr int bits(int stage) { return N - stage * DB - BB_; }
    static constexpr int words(int stage) { return (bits(stage) + 31) / 32; }
    static constexpr int WMAX = words(0);
    static constexpr size_t ROWS = (size_t)NBUCKETS * NSLOTS;
    static_assert(BB_ + 2 * SB_ <= 32, "parent reference must fit 32 bits");
    static_assert(NSLOTS_ <= (1 << SB_), "slot index must fit SLOTBITS");
    static_assert(DB < 32 && DB >= BB_, "digit geometry");
};

// Mainnet/testnet (200,9); test network (96,5); regtest (48,5).
using Cfg200_9 = EhCfg<200, 9, 12, 640, 10, 64>;
using Cfg96_5 = EhCfg<96, 5, 10, 256, 8, 64>;
using Cfg48_5 = EhCfg<48, 5, 4, 64, 6, 64>;

constexpr int NT = 256;
constexpr uint32_t NIL = 0xffffffffu;
constexpr int MAX_CHAIN = 64;

template <class C>
__device__ __forceinline__ uint32_t pack_ref(uint32_t b, uint32_t sa, uint32_t sb) {
    return (b << (2 * C::SLOTBITS)) | (sa << C::SLOTBITS) | sb;
}

// ------------------------------------------------------------------ stage 0
template <class C>
__global__ __launch_bounds__(NT) void eh_gen(const EhBaseState* __restrict__ states, uint32_t* __restrict__ hout,
                                             uint32_t* __restrict__ cnt0, uint32_t* __restrict__ ref0) {
    constexpr int W0 = C::words(0);
    constexpr int SW = (C::N + 31) / 32 + 1;
    const int nonce = blockIdx.y;
    const uint32_t g = blockIdx.x * NT + threadIdx.x;
    if (g >= (uint32_t)C::NHASH) return;
    uint64_t h[8];
    eh_hash_g(states[nonce], g, h);
#pragma unroll
    for (int s = 0; s < C::IPH; ++s) {
        const uint32_t idx = g * C::IPH + s;
        if (idx >= (uint32_t)C::INIT) break;
        uint32_t S[SW];
#pragma unroll
        for (int w = 0; w < SW; ++w) {
            uint32_t v = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int k = 4 * w + t;
                const uint32_t byte = (k < C::NBYTES) ? digest_byte(h, s * C::NBYTES + k) : 0u;
                v = (v << 8) | byte;
            }
            S[w] = v;
        }
        const uint32_t bucket = S[0] >> (32 - C::BUCKBITS);
        const uint32_t slot = atomicAdd(&cnt0[nonce * C::NBUCKETS + bucket], 1u);
        if (slot < (uint32_t)C::NSLOTS) {
            const size_t row = ((size_t)nonce * C::NBUCKETS + bucket) * C::NSLOTS + slot;
            uint32_t* dst = hout + row * W0;
#pragma unroll
            for (int w = 0; w < W0; ++w) dst[w] = (S[w] << C::BUCKBITS) | (S[w + 1] >> (32 - C::BUCKBITS));
            ref0[row] = idx;
        }
    }
}

// ------------------------------------------------------------------ stages 1..K
// STAGE < K: collision round producing stage-STAGE rows. STAGE == K: final round.
template <class C, int STAGE>
__global__ __launch_bounds__(NT) void eh_round(const uint32_t* __restrict__ hin, const uint32_t* __restrict__ cin,
                                               uint32_t* __restrict__ hout, uint32_t* __restrict__ cout,
                                               uint32_t* __restrict__ refout, uint32_t* __restrict__ ncand,
                                               uint32_t* __restrict__ cand) {
    constexpr int WI = C::words(STAGE - 1);
    constexpr int WO = (STAGE < C::K) ? C::words(STAGE) : 1;
    __shared__ uint32_t rows[C::NSLOTS * WI];
    __shared__ uint32_t nxt[C::NSLOTS];
    __shared__ uint32_t head[C::NRESTS];
    const uint32_t b = blockIdx.x % C::NBUCKETS;
    const uint32_t nonce = blockIdx.x / C::NBUCKETS;
    const uint32_t tid = threadIdx.x;
    const uint32_t n = min(cin[nonce * C::NBUCKETS + b], (uint32_t)C::NSLOTS);
    const uint32_t* src = hin + ((size_t)nonce * C::NBUCKETS + b) * C::NSLOTS * WI;
    for (uint32_t k = tid; k < n * WI; k += NT) rows[k] = src[k];
    for (uint32_t k = tid; k < (uint32_t)C::NRESTS; k += NT) head[k] = NIL;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += NT) {
        const uint32_t key = (C::RESTBITS > 0) ? (rows[i * WI] >> ((32 - C::RESTBITS) & 31)) : 0u;
        nxt[i] = atomicExch(&head[key], i);
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += NT) {
        uint32_t ri[WI];
#pragma unroll
        for (int w = 0; w < WI; ++w) ri[w] = rows[i * WI + w];
        int steps = 0;
        for (uint32_t j = nxt[i]; j != NIL && steps < MAX_CHAIN; j = nxt[j], ++steps) {
            uint32_t x[WI + 1];
            uint32_t any = 0;
#pragma unroll
            for (int w = 0; w < WI; ++w) {
                x[w] = ri[w] ^ rows[j * WI + w];
                any |= x[w];
            }
            x[WI] = 0;
            if constexpr (STAGE < C::K) {
                if (any == 0) continue; // identical subtrees: duplicate indices
                const uint32_t nb = (x[0] >> (32 - C::DB)) & (C::NBUCKETS - 1);
                const uint32_t slot = atomicAdd(&cout[nonce * C::NBUCKETS + nb], 1u);
                if (slot < (uint32_t)C::NSLOTS) {
                    const size_t row = ((size_t)nonce * C::NBUCKETS + nb) * C::NSLOTS + slot;
                    uint32_t* dst = hout + row * WO;
#pragma unroll
                    for (int w = 0; w < WO; ++w) dst[w] = (x[w] << C::DB) | (x[w + 1] >> (32 - C::DB));
                    refout[row] = pack_ref<C>(b, j, i);
                }
            } else {
                if (any == 0) {
                    const uint32_t c = atomicAdd(&ncand[nonce], 1u);
                    if (c < (uint32_t)C::MAXCAND) cand[nonce * C::MAXCAND + c] = pack_ref<C>(b, j, i);
                }
            }
        }
    }
}

// ------------------------------------------------------------------ tree expansion
// refs: K arrays of B*ROWS parent references (stage 0 holds leaf indices).
template <class C>
__global__ __launch_bounds__(C::L < 64 ? 64 : C::L) void eh_expand(const uint32_t* __restrict__ refs,
                                                                  const uint32_t* __restrict__ ncand,
                                                                  const uint32_t* __restrict__ cand, int batch,
                                                                  uint32_t* __restrict__ out_idx,
                                                                  uint32_t* __restrict__ out_valid) {
    constexpr int L = C::L;
    __shared__ uint32_t buf[2][L];
    __shared__ uint32_t dup;
    const uint32_t c = blockIdx.x % C::MAXCAND;
    const uint32_t nonce = blockIdx.x / C::MAXCAND;
    const uint32_t t = threadIdx.x;
    const uint32_t nc = min(ncand[nonce], (uint32_t)C::MAXCAND);
    if (c >= nc) return; // uniform per workgroup
    if (t == 0) {
        buf[0][0] = cand[nonce * C::MAXCAND + c];
        dup = 0;
    }
    int cur = 0;
    for (int s = C::K; s >= 1; --s) {
        __syncthreads();
        const uint32_t cnt = 1u << (C::K - s); // nodes at this level
        if (t < 2 * cnt) {
            const uint32_t p = buf[cur][t >> 1];
            const uint32_t bk = p >> (2 * C::SLOTBITS);
            const uint32_t slot = (t & 1) ? (p & C::SLOTMASK) : ((p >> C::SLOTBITS) & C::SLOTMASK);
            const uint32_t* R = refs + (size_t)(s - 1) * batch * C::ROWS + (size_t)nonce * C::ROWS;
            buf[cur ^ 1][t] = R[(size_t)bk * C::NSLOTS + slot];
        }
        cur ^= 1;
    }
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
    DevBuf<uint32_t> d_hash[2], d_refs, d_cnt, d_ncand, d_cand, d_idx, d_valid;
    HostBuf<bcpk::EhBaseState> h_states;
    HostBuf<uint32_t> h_ncand, h_idx, h_valid, h_cnt_sample;
    size_t rows = 0, L = 0, maxcand = 0, nbuckets = 0, kstages = 0, cnt_words = 0;
    int inflight = 0;
    EhGpuStats stats;
    size_t bytes = 0;

    template <class C> void alloc() {
        rows = C::ROWS;
        L = C::L;
        maxcand = C::MAXCAND;
        nbuckets = C::NBUCKETS;
        kstages = C::K;
        d_states.alloc(batch);
        h_states.alloc(batch);
        d_hash[0].alloc((size_t)batch * C::ROWS * C::WMAX);
        d_hash[1].alloc((size_t)batch * C::ROWS * C::WMAX);
        d_refs.alloc((size_t)C::K * batch * C::ROWS);
        cnt_words = (size_t)C::K * batch * C::NBUCKETS + batch; // + ncand
        d_cnt.alloc(cnt_words);
        d_cand.alloc((size_t)batch * C::MAXCAND);
        d_idx.alloc((size_t)batch * C::MAXCAND * C::L);
        d_valid.alloc((size_t)batch * C::MAXCAND);
        h_ncand.alloc(batch);
        h_idx.alloc((size_t)batch * C::MAXCAND * C::L);
        h_valid.alloc((size_t)batch * C::MAXCAND);
        h_cnt_sample.alloc(C::NBUCKETS);
        bytes = 2 * d_hash[0].n * 4 + d_refs.n * 4 + d_cnt.n * 4 + d_idx.n * 4;
    }

    template <class C, int S> void launch_round(uint32_t* cnt, uint32_t* ncand) {
        const uint32_t* hin = d_hash[(S - 1) & 1].p;
        uint32_t* hout = d_hash[S & 1].p;
        const uint32_t* cin = cnt + (size_t)(S - 1) * batch * C::NBUCKETS;
        uint32_t* cout = (S < C::K) ? cnt + (size_t)S * batch * C::NBUCKETS : nullptr;
        uint32_t* refout = (S < C::K) ? d_refs.p + (size_t)S * batch * C::ROWS : nullptr;
        hipLaunchKernelGGL((bcpk::eh_round<C, S>), dim3(C::NBUCKETS * batch), dim3(bcpk::NT), 0, stream, hin, cin,
                           hout, cout, refout, ncand, d_cand.p);
    }
    template <class C, int... S> void launch_rounds(uint32_t* cnt, uint32_t* ncand, std::integer_sequence<int, S...>) {
        (launch_round<C, S + 1>(cnt, ncand), ...);
    }

    template <class C> void launch(size_t nstates) {
        uint32_t* cnt = d_cnt.p;
        uint32_t* ncand = d_cnt.p + (size_t)C::K * batch * C::NBUCKETS;
        BCP_HIP_CHECK(hipMemcpyAsync(d_states.p, h_states.p, nstates * sizeof(bcpk::EhBaseState),
                                     hipMemcpyHostToDevice, stream));
        BCP_HIP_CHECK(hipMemsetAsync(d_cnt.p, 0, d_cnt.n * sizeof(uint32_t), stream));
        BCP_HIP_CHECK(hipEventRecord(ev0, stream));
        hipLaunchKernelGGL((bcpk::eh_gen<C>), dim3((C::NHASH + bcpk::NT - 1) / bcpk::NT, nstates), dim3(bcpk::NT), 0,
                           stream, d_states.p, d_hash[0].p, cnt, d_refs.p);
        launch_rounds<C>(cnt, ncand, std::make_integer_sequence<int, C::K>{});
        constexpr int EB = C::L < 64 ? 64 : C::L;
        hipLaunchKernelGGL((bcpk::eh_expand<C>), dim3(C::MAXCAND * nstates), dim3(EB), 0, stream, d_refs.p, ncand,
                           d_cand.p, batch, d_idx.p, d_valid.p);
        BCP_HIP_CHECK(hipGetLastError());
        BCP_HIP_CHECK(hipEventRecord(ev1, stream));
        BCP_HIP_CHECK(hipMemcpyAsync(h_ncand.p, ncand, nstates * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        BCP_HIP_CHECK(hipMemcpyAsync(h_valid.p, d_valid.p, nstates * C::MAXCAND * sizeof(uint32_t),
                                     hipMemcpyDeviceToHost, stream));
        BCP_HIP_CHECK(hipMemcpyAsync(h_idx.p, d_idx.p, nstates * C::MAXCAND * C::L * sizeof(uint32_t),
                                     hipMemcpyDeviceToHost, stream));
        // Sample the last collision round's bucket fill of nonce 0 for overflow accounting.
        BCP_HIP_CHECK(hipMemcpyAsync(h_cnt_sample.p, cnt + (size_t)(C::K - 1) * batch * C::NBUCKETS,
                                     C::NBUCKETS * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
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
void EquihashGpuSolver::ResetStats() { impl->stats = EhGpuStats(); }
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
    for (size_t bkt = 0; bkt < impl->nbuckets; ++bkt) {
        uint32_t c = impl->h_cnt_sample.p[bkt];
        // NSLOTS is encoded in rows / nbuckets
        uint32_t cap = (uint32_t)(impl->rows / impl->nbuckets);
        if (c > cap) impl->stats.dropped_rows += c - cap;
    }
    std::vector<std::vector<std::vector<uint32_t>>> out(ns);
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
