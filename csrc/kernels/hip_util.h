// Small host helpers shared by the .hip translation units.
#pragma once
#include <hip/hip_runtime.h>

#include "kernels/gpu_api.h"

#include <stdexcept>
#include <string>

#define BCP_HIP_CHECK(expr)                                                                            \
    do {                                                                                               \
        hipError_t _e = (expr);                                                                        \
        if (_e != hipSuccess)                                                                          \
            throw std::runtime_error(std::string("HIP error in ") + #expr + ": " + hipGetErrorString(_e) + \
                                     " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")");          \
    } while (0)

namespace bcp {
namespace gpu {

// Resolves -1 to the caller's current device and makes `device` current.
inline int UseDevice(int device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        throw std::runtime_error("bitcoincashplus_amd: no HIP device available (gfx950 kernels need an MI355X)");
    if (device < 0) BCP_HIP_CHECK(hipGetDevice(&device));
    if (device >= count) throw std::runtime_error("bitcoincashplus_amd: device index out of range");
    BCP_HIP_CHECK(hipSetDevice(device));
    return device;
}

// Makes `device` (-1: the current one) current for a scope and restores the caller's device
// after: the device-resident entry points run on threads (torch's) whose current device matters.
struct DeviceScope {
    int prev = -1;
    int device = -1;
    explicit DeviceScope(int d) {
        BCP_HIP_CHECK(hipGetDevice(&prev));
        device = UseDevice(d);
    }
    ~DeviceScope() {
        if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

// RAII device buffer.
template <typename T> struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() {}
    explicit DevBuf(size_t count) { alloc(count); }
    void alloc(size_t count) {
        release();
        n = count;
        if (count) BCP_HIP_CHECK(hipMalloc((void**)&p, count * sizeof(T)));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DevBuf() { release(); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
};

// RAII pinned host buffer.
template <typename T> struct HostBuf {
    T* p = nullptr;
    size_t n = 0;
    void alloc(size_t count) {
        release();
        n = count;
        if (count) BCP_HIP_CHECK(hipHostMalloc((void**)&p, count * sizeof(T), hipHostMallocDefault));
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
    ~HostBuf() { release(); }
};

// Per-lane execution state (VerifyLane::Impl, gpu_api.h): a stream and grow-only staging.
// Slots index independent buffers so one batch can stage several arrays.
struct LaneState {
    int device = 0;
    int priority = 0;
    hipStream_t stream = nullptr;
    static constexpr int SLOTS = 4;
    HostBuf<unsigned char> host[SLOTS];
    DevBuf<unsigned char> dev[SLOTS];
    uint64_t batches = 0, items = 0;
    // host share (the caller's fill into pinned staging) and device share (copies, kernels and
    // the wait for them) of the batches, microseconds
    uint64_t fillMicros = 0, deviceMicros = 0;
    unsigned char* Host(int slot, size_t bytes) {
        if (host[slot].n < bytes) host[slot].alloc(bytes + bytes / 2);
        return host[slot].p;
    }
    unsigned char* Dev(int slot, size_t bytes) {
        if (dev[slot].n < bytes) dev[slot].alloc(bytes + bytes / 2);
        return dev[slot].p;
    }
};

struct VerifyLane::Impl : LaneState {};

} // namespace gpu
} // namespace bcp
