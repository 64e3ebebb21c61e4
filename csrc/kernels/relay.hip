// Relay-path batch kernels for CDNA4:
//   K9  BIP152 short transaction ids (SipHash-2-4 of a txid, 48 bits): the mempool side of
//       compact-block reconstruction, reference src/blockencodings.cpp:37-42 and
//       PartiallyDownloadedBlock::InitData (:67-178), SipHashUint256 src/hash.cpp:181-300;
// One lane per item; 64-bit SipHash words stay in VGPR pairs (v_lshl_add_u64 adds,
// v_alignbit rotates).
#include <hip/hip_runtime.h>

#include "kernels/gpu_api.h"
#include "kernels/hip_util.h"

#include <algorithm>
#include <cstring>
#include <mutex>
#include <stdexcept>

namespace bcpk {

__device__ __forceinline__ uint64_t rotl64d(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }

#define BCP_SIPROUND                                                                                   \
    do {                                                                                               \
        v0 += v1; v1 = rotl64d(v1, 13); v1 ^= v0; v0 = rotl64d(v0, 32);                                \
        v2 += v3; v3 = rotl64d(v3, 16); v3 ^= v2;                                                      \
        v0 += v3; v3 = rotl64d(v3, 21); v3 ^= v0;                                                      \
        v2 += v1; v1 = rotl64d(v1, 17); v1 ^= v2; v2 = rotl64d(v2, 32);                                \
    } while (0)

__global__ __launch_bounds__(256) void shortid_kernel(uint64_t k0, uint64_t k1, const uint4* __restrict__ txids,
                                                      uint64_t* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 a = txids[2 * i], b = txids[2 * i + 1];
    const uint64_t d[4] = {((uint64_t)a.y << 32) | a.x, ((uint64_t)a.w << 32) | a.z, ((uint64_t)b.y << 32) | b.x,
                           ((uint64_t)b.w << 32) | b.z};
    uint64_t v0 = 0x736f6d6570736575ULL ^ k0, v1 = 0x646f72616e646f6dULL ^ k1;
    uint64_t v2 = 0x6c7967656e657261ULL ^ k0, v3 = 0x7465646279746573ULL ^ k1;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        v3 ^= d[w];
        BCP_SIPROUND;
        BCP_SIPROUND;
        v0 ^= d[w];
    }
    const uint64_t t = 32ULL << 56; // message length 32 bytes, no tail bytes
    v3 ^= t;
    BCP_SIPROUND;
    BCP_SIPROUND;
    v0 ^= t;
    v2 ^= 0xff;
    BCP_SIPROUND;
    BCP_SIPROUND;
    BCP_SIPROUND;
    BCP_SIPROUND;
    out[i] = (v0 ^ v1 ^ v2 ^ v3) & 0xffffffffffffULL;
}
#undef BCP_SIPROUND

} // namespace bcpk

namespace bcp {
namespace gpu {

namespace {
// Per-device stream and grow-only pinned/device staging of the relay entry points; calls on
// one device are serialised by its mutex.
struct RelayCtx {
    std::mutex m;
    hipStream_t s = nullptr;
    LaneState st; // staging slots only (the stream above is the one used)
};
RelayCtx& Ctx(int device) {
    static RelayCtx ctx[64];
    if (device < 0 || device >= 64) throw std::runtime_error("relay GPU context: device index out of range");
    return ctx[device];
}
std::unique_lock<std::mutex> Lock(RelayCtx& c) {
    std::unique_lock<std::mutex> l(c.m);
    if (!c.s) BCP_HIP_CHECK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
    return l;
}
} // namespace

std::vector<uint64_t> ShortTxIdBatch(uint64_t k0, uint64_t k1, const unsigned char* txids32, size_t n, int device) {
    std::vector<uint64_t> out(n);
    if (!n) return out;
    device = UseDevice(device);
    RelayCtx& c = Ctx(device);
    auto l = Lock(c);
    unsigned char* h_in = c.st.Host(0, n * 32);
    unsigned char* h_out = c.st.Host(1, n * 8);
    unsigned char* d_in = c.st.Dev(0, n * 32);
    unsigned char* d_out = c.st.Dev(1, n * 8);
    memcpy(h_in, txids32, n * 32);
    BCP_HIP_CHECK(hipMemcpyAsync(d_in, h_in, n * 32, hipMemcpyHostToDevice, c.s));
    hipLaunchKernelGGL(bcpk::shortid_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c.s, k0, k1,
                       reinterpret_cast<const uint4*>(d_in), reinterpret_cast<uint64_t*>(d_out), n);
    BCP_HIP_CHECK(hipGetLastError());
    BCP_HIP_CHECK(hipMemcpyAsync(h_out, d_out, n * 8, hipMemcpyDeviceToHost, c.s));
    BCP_HIP_CHECK(hipStreamSynchronize(c.s));
    memcpy(out.data(), h_out, n * 8);
    return out;
}

void ShortTxIdsDevice(uint64_t k0, uint64_t k1, const void* txids32, void* out64, size_t n, int device,
                      uintptr_t stream) {
    if (!n) return;
    if (reinterpret_cast<uintptr_t>(txids32) % 16) throw std::invalid_argument("ShortTxIdsDevice: txids not 16-byte aligned");
    DeviceScope ds(device);
    hipLaunchKernelGGL(bcpk::shortid_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), k0, k1, static_cast<const uint4*>(txids32),
                       static_cast<uint64_t*>(out64), n);
    BCP_HIP_CHECK(hipGetLastError());
}

} // namespace gpu
} // namespace bcp
