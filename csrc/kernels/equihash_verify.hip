// Batched Equihash consensus verification on CDNA4 — the GPU form of reference
// Equihash<N,K>::IsValidSolution (src/crypto/equihash.cpp:725-770), called per
// header from CheckEquihashSolution (src/pow.cpp:298) on every header accept,
// headers message (<= 2000, src/validation.h:101) and block read.
//
// One workgroup per solution, one lane per leaf (2^K lanes):
//   1. lane t decodes index t from the (CBL+1)-bit big-endian minimal encoding,
//   2. hashes H(base || le32(idx / IPH)) and keeps slice idx % IPH as a bit string,
//   3. K LDS tree levels: collision on digit l, subtree order (left first index <
//      right first index), XOR; the root's last digit must be zero,
//   4. distinctness of all 2^K indices via an LDS bitonic sort.
// The boolean equals the reference's: every reference rejection reason maps to
// one of these checks (order-of-checks only changes which reason, not the result).
#include <hip/hip_runtime.h>

#include <chrono>

#include "kernels/blake2b_device.h"
#include "kernels/gpu_api.h"
#include "kernels/hip_util.h"

#include <cstring>
#include <memory>
#include <mutex>

#include <cstring>
#include <stdexcept>

namespace bcpk {

template <int N_, int K_> struct EvCfg {
    static constexpr int N = N_, K = K_;
    static constexpr int DB = N / (K + 1);
    static constexpr int IPH = 512 / N;
    static constexpr int NBYTES = N / 8;
    static constexpr int L = 1 << K;
    static constexpr int SW = (N + 31) / 32; // stream words
    static constexpr int SOLW = L * (DB + 1) / 8;
    static constexpr int NTH = L < 64 ? 64 : L;
};

template <class C> __device__ __forceinline__ uint32_t stream_bits(const uint32_t* S, int bit0, int nbits) {
    // nbits <= 25; may straddle two words.
    const int w = bit0 >> 5, o = bit0 & 31;
    uint64_t v = ((uint64_t)S[w] << 32) | (w + 1 < C::SW ? S[w + 1] : 0u);
    return (uint32_t)(v >> (64 - o - nbits)) & ((1u << nbits) - 1);
}

template <class C>
__global__ __launch_bounds__(C::NTH) void eh_verify(const EhBaseState* __restrict__ states,
                                                   const uint8_t* __restrict__ sols, uint8_t* __restrict__ ok) {
    constexpr int L = C::L, SW = C::SW;
    __shared__ uint32_t S[L][SW + 1];
    __shared__ uint32_t first[L];
    __shared__ uint32_t srt[L];
    __shared__ uint32_t bad;
    const int item = blockIdx.x;
    const int t = threadIdx.x;
    if (t == 0) bad = 0;
    const uint8_t* sol = sols + (size_t)item * C::SOLW;
    uint32_t idx = 0;
    if (t < L) {
        // index t occupies bits [t*(DB+1), (t+1)*(DB+1)) of the big-endian minimal encoding
        const int nb = C::DB + 1;
        const int bit0 = t * nb;
        const int byte0 = bit0 >> 3;
        uint64_t v = 0;
#pragma unroll
        for (int q = 0; q < 5; ++q) v = (v << 8) | ((byte0 + q < C::SOLW) ? sol[byte0 + q] : 0u);
        idx = (uint32_t)(v >> (40 - (bit0 & 7) - nb)) & ((1u << nb) - 1);
        uint64_t h[8];
        eh_hash_g(states[item], idx / C::IPH, h);
        const int sel = idx % C::IPH;
        uint32_t st[SW];
#pragma unroll
        for (int w = 0; w < SW; ++w) st[w] = 0;
#pragma unroll
        for (int s = 0; s < C::IPH; ++s) {
            if (s == sel) {
#pragma unroll
                for (int w = 0; w < SW; ++w) {
                    uint32_t v32 = 0;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int k = 4 * w + q;
                        v32 = (v32 << 8) | ((k < C::NBYTES) ? digest_byte(h, s * C::NBYTES + k) : 0u);
                    }
                    st[w] = v32;
                }
            }
        }
#pragma unroll
        for (int w = 0; w < SW; ++w) S[t][w] = st[w];
        S[t][SW] = 0;
        first[t] = idx;
        srt[t] = idx;
    }
    for (int l = 0; l < C::K; ++l) {
        __syncthreads();
        const int w = 1 << l;
        if (t < L && (t & (2 * w - 1)) == 0) {
            const int a = t, b = t + w;
            const uint32_t da = stream_bits<C>(S[a], l * C::DB, C::DB);
            const uint32_t db = stream_bits<C>(S[b], l * C::DB, C::DB);
            if (da != db) atomicOr(&bad, 1u);
            if (!(first[a] < first[b])) atomicOr(&bad, 2u);
#pragma unroll
            for (int q = 0; q < SW; ++q) S[a][q] ^= S[b][q];
        }
    }
    // distinct indices
    for (uint32_t k = 2; k <= (uint32_t)L; k <<= 1) {
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            __syncthreads();
            if (t < L) {
                const uint32_t ixj = t ^ jj;
                if (ixj > (uint32_t)t) {
                    const uint32_t a = srt[t], b = srt[ixj];
                    const bool up = (t & k) == 0;
                    if ((a > b) == up) {
                        srt[t] = b;
                        srt[ixj] = a;
                    }
                }
            }
        }
    }
    __syncthreads();
    if (t + 1 < L && srt[t] == srt[t + 1]) atomicOr(&bad, 4u);
    if (t == 0 && stream_bits<C>(S[0], C::K * C::DB, C::DB) != 0) atomicOr(&bad, 8u);
    __syncthreads();
    if (t == 0) ok[item] = bad ? 0 : 1;
}

// One lane per header: the base state from the raw 140-byte Equihash input (header prep on the
// device instead of a host BLAKE2b per header).
__global__ __launch_bounds__(64) void eh_state_kernel(const uint8_t* __restrict__ in140, EhBaseState* __restrict__ out,
                                                      uint32_t N, uint32_t K, int n) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    EhBaseState bs;
    eh_header_state(in140 + (size_t)i * 140, N, K, bs);
    out[i] = bs;
}

} // namespace bcpk

namespace bcp {
namespace gpu {

// Stages n (state, solution) pairs through the lane's pinned buffers: one H2D copy of the
// packed states + solutions, one kernel (one workgroup per solution), one D2H copy.
template <class C>
static void verify_lane(LaneState& L, const EhBaseState* states, const std::vector<unsigned char>* const* sols,
                        size_t n, uint8_t* result) {
    if (n == 0) return;
    BCP_HIP_CHECK(hipSetDevice(L.device));
    const size_t sb = n * sizeof(EhBaseState), pb = n * C::SOLW;
    unsigned char* h_in = L.Host(0, sb + pb);
    uint8_t* h_ok = L.Host(1, n);
    memcpy(h_in, states, sb);
    std::vector<char> lenok(n, 0);
    for (size_t i = 0; i < n; ++i) {
        unsigned char* dst = h_in + sb + i * C::SOLW;
        if (sols[i]->size() == (size_t)C::SOLW) {
            memcpy(dst, sols[i]->data(), C::SOLW);
            lenok[i] = 1;
        } else {
            memset(dst, 0, C::SOLW);
        }
    }
    unsigned char* d_in = L.Dev(0, sb + pb);
    uint8_t* d_ok = L.Dev(1, n);
    BCP_HIP_CHECK(hipMemcpyAsync(d_in, h_in, sb + pb, hipMemcpyHostToDevice, L.stream));
    hipLaunchKernelGGL((bcpk::eh_verify<C>), dim3(n), dim3(C::NTH), 0, L.stream,
                       reinterpret_cast<const bcpk::EhBaseState*>(d_in), (const uint8_t*)(d_in + sb), d_ok);
    BCP_HIP_CHECK(hipGetLastError());
    BCP_HIP_CHECK(hipMemcpyAsync(h_ok, d_ok, n, hipMemcpyDeviceToHost, L.stream));
    BCP_HIP_CHECK(hipStreamSynchronize(L.stream));
    for (size_t i = 0; i < n; ++i) result[i] = lenok[i] ? h_ok[i] : 0; // reference: invalid solution length
    L.batches++;
    L.items += n;
}

// Raw headers: `fill` writes n x 140 input bytes, n x SOLW solution bytes and n length flags
// straight into the pinned staging; one H2D copy, the state kernel, the verify kernel, one D2H.
template <class C>
static void verify_lane_headers(LaneState& L, size_t n, const std::function<void(uint8_t*, uint8_t*, uint8_t*)>& fill,
                                uint8_t* result) {
    if (n == 0) return;
    BCP_HIP_CHECK(hipSetDevice(L.device));
    const size_t ib = (n * 140 + 15) & ~(size_t)15, pb = n * C::SOLW;
    unsigned char* h_in = L.Host(0, ib + pb + n);
    uint8_t* lenok = h_in + ib + pb;
    const auto t0 = std::chrono::steady_clock::now();
    fill(h_in, h_in + ib, lenok);
    const auto t1 = std::chrono::steady_clock::now();
    uint8_t* h_ok = L.Host(1, n);
    unsigned char* d_in = L.Dev(0, ib + pb);
    bcpk::EhBaseState* d_states = reinterpret_cast<bcpk::EhBaseState*>(L.Dev(2, n * sizeof(bcpk::EhBaseState)));
    uint8_t* d_ok = L.Dev(1, n);
    BCP_HIP_CHECK(hipMemcpyAsync(d_in, h_in, ib + pb, hipMemcpyHostToDevice, L.stream));
    hipLaunchKernelGGL(bcpk::eh_state_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, L.stream,
                       (const uint8_t*)d_in, d_states, (uint32_t)C::N, (uint32_t)C::K, (int)n);
    BCP_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL((bcpk::eh_verify<C>), dim3(n), dim3(C::NTH), 0, L.stream, (const bcpk::EhBaseState*)d_states,
                       (const uint8_t*)(d_in + ib), d_ok);
    BCP_HIP_CHECK(hipGetLastError());
    BCP_HIP_CHECK(hipMemcpyAsync(h_ok, d_ok, n, hipMemcpyDeviceToHost, L.stream));
    BCP_HIP_CHECK(hipStreamSynchronize(L.stream));
    for (size_t i = 0; i < n; ++i) result[i] = lenok[i] ? h_ok[i] : 0;
    const auto t2 = std::chrono::steady_clock::now();
    L.fillMicros += std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
    L.deviceMicros += std::chrono::duration_cast<std::chrono::microseconds>(t2 - t1).count();
    L.batches++;
    L.items += n;
}

void VerifyLane::EquihashHeaders(unsigned N, unsigned K, size_t n,
                                 const std::function<void(uint8_t*, uint8_t*, uint8_t*)>& fill, uint8_t* result) {
    if (N == 200 && K == 9) return verify_lane_headers<bcpk::EvCfg<200, 9>>(*impl, n, fill, result);
    if (N == 96 && K == 5) return verify_lane_headers<bcpk::EvCfg<96, 5>>(*impl, n, fill, result);
    if (N == 48 && K == 5) return verify_lane_headers<bcpk::EvCfg<48, 5>>(*impl, n, fill, result);
    if (N == 96 && K == 3) return verify_lane_headers<bcpk::EvCfg<96, 3>>(*impl, n, fill, result);
    throw std::invalid_argument("EquihashVerifyBatch: unsupported (N,K)");
}

size_t EquihashSolutionBytes(unsigned N, unsigned K) { return ((size_t)1 << K) * (N / (K + 1) + 1) / 8; }

VerifyLane::VerifyLane(int device, bool highPriority) : impl(new Impl) {
    impl->device = UseDevice(device);
    int least = 0, greatest = 0;
    BCP_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    impl->priority = highPriority ? greatest : least;
    BCP_HIP_CHECK(hipStreamCreateWithPriority(&impl->stream, hipStreamNonBlocking, impl->priority));
}
VerifyLane::~VerifyLane() {
    if (impl && impl->stream) {
        (void)hipSetDevice(impl->device);
        (void)hipStreamSynchronize(impl->stream);
        (void)hipStreamDestroy(impl->stream);
    }
}
int VerifyLane::Device() const { return impl->device; }
int VerifyLane::Priority() const { return impl->priority; }
uint64_t VerifyLane::Batches() const { return impl->batches; }
uint64_t VerifyLane::Items() const { return impl->items; }
uint64_t VerifyLane::FillMicros() const { return impl->fillMicros; }
uint64_t VerifyLane::DeviceMicros() const { return impl->deviceMicros; }

void VerifyLane::Equihash(unsigned N, unsigned K, const EhBaseState* states,
                          const std::vector<unsigned char>* const* sols, size_t n, uint8_t* result) {
    if (N == 200 && K == 9) return verify_lane<bcpk::EvCfg<200, 9>>(*impl, states, sols, n, result);
    if (N == 96 && K == 5) return verify_lane<bcpk::EvCfg<96, 5>>(*impl, states, sols, n, result);
    if (N == 48 && K == 5) return verify_lane<bcpk::EvCfg<48, 5>>(*impl, states, sols, n, result);
    if (N == 96 && K == 3) return verify_lane<bcpk::EvCfg<96, 3>>(*impl, states, sols, n, result);
    throw std::invalid_argument("EquihashVerifyBatch: unsupported (N,K)");
}

// One default (normal-priority) lane per device for the plain batch API.
static VerifyLane& DefaultLane(int device, std::unique_lock<std::mutex>& hold) {
    static std::mutex m;
    static std::unique_ptr<VerifyLane> lanes[64];
    static std::mutex use[64];
    const int dev = UseDevice(device);
    if (dev >= 64) throw std::runtime_error("device index out of range");
    {
        std::lock_guard<std::mutex> l(m);
        if (!lanes[dev]) lanes[dev].reset(new VerifyLane(dev, false));
    }
    hold = std::unique_lock<std::mutex>(use[dev]);
    return *lanes[dev];
}

std::vector<uint8_t> EquihashVerifyBatch(unsigned n, unsigned k, const std::vector<EhBaseState>& states,
                                         const std::vector<std::vector<unsigned char>>& solutions, int device) {
    if (states.size() != solutions.size()) throw std::invalid_argument("states/solutions size mismatch");
    std::vector<uint8_t> result(states.size(), 0);
    if (states.empty()) return result;
    std::vector<const std::vector<unsigned char>*> ptrs(solutions.size());
    for (size_t i = 0; i < solutions.size(); ++i) ptrs[i] = &solutions[i];
    std::unique_lock<std::mutex> hold;
    VerifyLane& lane = DefaultLane(device, hold);
    lane.Equihash(n, k, states.data(), ptrs.data(), states.size(), result.data());
    return result;
}

bool GpuAvailable() {
    // asked per block (and per batch): probe the runtime once, devices do not come and go
    static const bool available = [] {
        int count = 0;
        return hipGetDeviceCount(&count) == hipSuccess && count > 0;
    }();
    return available;
}

int DeviceCount() {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return 0;
    return count;
}

std::string DeviceName(int device) {
    hipDeviceProp_t prop;
    BCP_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    return std::string(prop.name) + " (" + prop.gcnArchName + ", " + std::to_string(prop.multiProcessorCount) + " CUs)";
}

void Check(int st, const char* what) {
    if (st != hipSuccess)
        throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString((hipError_t)st));
}

} // namespace gpu
} // namespace bcp
