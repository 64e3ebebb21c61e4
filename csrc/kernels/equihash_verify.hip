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

#include "kernels/blake2b_device.h"
#include "kernels/gpu_api.h"
#include "kernels/hip_util.h"

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

} // namespace bcpk

namespace bcp {
namespace gpu {

template <class C>
static std::vector<uint8_t> verify_impl(const std::vector<EhBaseState>& states,
                                        const std::vector<std::vector<unsigned char>>& sols, int device) {
    UseDevice(device);
    const size_t n = states.size();
    std::vector<uint8_t> result(n, 0);
    if (n == 0) return result;
    std::vector<uint8_t> packed(n * C::SOLW, 0);
    std::vector<char> lenok(n, 0);
    for (size_t i = 0; i < n; ++i) {
        if (sols[i].size() == (size_t)C::SOLW) {
            memcpy(&packed[i * C::SOLW], sols[i].data(), C::SOLW);
            lenok[i] = 1;
        }
    }
    DevBuf<bcpk::EhBaseState> d_states(n);
    DevBuf<uint8_t> d_sols(packed.size()), d_ok(n);
    hipStream_t s;
    BCP_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    BCP_HIP_CHECK(hipMemcpyAsync(d_states.p, states.data(), n * sizeof(EhBaseState), hipMemcpyHostToDevice, s));
    BCP_HIP_CHECK(hipMemcpyAsync(d_sols.p, packed.data(), packed.size(), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL((bcpk::eh_verify<C>), dim3(n), dim3(C::NTH), 0, s, d_states.p, d_sols.p, d_ok.p);
    BCP_HIP_CHECK(hipGetLastError());
    BCP_HIP_CHECK(hipMemcpyAsync(result.data(), d_ok.p, n, hipMemcpyDeviceToHost, s));
    BCP_HIP_CHECK(hipStreamSynchronize(s));
    BCP_HIP_CHECK(hipStreamDestroy(s));
    for (size_t i = 0; i < n; ++i)
        if (!lenok[i]) result[i] = 0; // reference: invalid solution length
    return result;
}

std::vector<uint8_t> EquihashVerifyBatch(unsigned n, unsigned k, const std::vector<EhBaseState>& states,
                                         const std::vector<std::vector<unsigned char>>& solutions, int device) {
    if (states.size() != solutions.size()) throw std::invalid_argument("states/solutions size mismatch");
    if (n == 200 && k == 9) return verify_impl<bcpk::EvCfg<200, 9>>(states, solutions, device);
    if (n == 96 && k == 5) return verify_impl<bcpk::EvCfg<96, 5>>(states, solutions, device);
    if (n == 48 && k == 5) return verify_impl<bcpk::EvCfg<48, 5>>(states, solutions, device);
    if (n == 96 && k == 3) return verify_impl<bcpk::EvCfg<96, 3>>(states, solutions, device);
    throw std::invalid_argument("EquihashVerifyBatch: unsupported (N,K)");
}

bool GpuAvailable() {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return false;
    return count > 0;
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
