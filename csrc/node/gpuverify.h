// GPU verification service: the node's validation batches (ECDSA signatures of a block, the
// Equihash solutions of a HEADERS message) sharded across the node's validation GPUs.
//
// Parity: reference src/checkqueue.h:27-164 (CCheckQueue: the master splits a block's script
// checks across -par threads and AND-reduces the verdicts) and src/validation.cpp:2011-2127
// (ConnectBlock's control.Add / control.Wait). The MI355X equivalent:
//  * one service thread per lane owns the lane's HIP stream (created at the device's greatest
//    stream priority, so a validation batch is scheduled ahead of the miner's persistent solver
//    kernels on a shared device) and its pinned staging buffers (gpu::VerifyLane);
//  * a batch is split into contiguous shards, one per lane, that run concurrently on their
//    devices; per-item verdicts are gathered in order (the caller AND-reduces);
//  * -gpuvalidationdevices selects the devices (default: every visible device, two lanes each); the built-in
//    miner leaves configured validation devices alone whenever other GPUs are available
//    (miner.cpp GetMinerGpuDevices);
//  * a lane failure fails the whole call (the caller re-verifies on the CPU: a device fault
//    must never decide validity);
//  * each lane has its own host-fill workers (a share of the cores), so the shards' host
//    preparation (DER parse, key forms, header bytes) runs concurrently instead of queueing on
//    one pool.
// A device may be listed twice (two lanes on one GPU, two streams): the test suite uses that
// to exercise the sharded path on a one-GPU box.
#pragma once
#include "kernels/gpu_api.h"
#include "util/util.h"

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace bcp {

// One shard of a batch: items [lo, hi) on lane `lane`.
struct VerifyShard {
    size_t lane, lo, hi;
};
// The shard plan of an n-item batch over lanes whose devices are laneDevices[i] (a device may
// own several lanes). Distinct devices are used first: the batch is cut into
// k = clamp(n / minPerDevice, 1, #devices) device shares (devices in first-listed order), and a
// device's share is spread over its further lanes only while each keeps >= minPerLane items
// (two kernels on one device do not overlap, so a second lane there pays only for very large
// batches). Shards are contiguous, in lane order, and sized evenly. Pure: no GPU needed.
std::vector<VerifyShard> PlanShards(size_t n, const std::vector<int>& laneDevices, size_t minPerDevice,
                                    size_t minPerLane);

class GpuVerifyService {
public:
    static GpuVerifyService& Instance();
    ~GpuVerifyService();

    // Validation devices (duplicates allowed: one lane each). Empty = default (every visible
    // device, twice). Takes effect for the next batch; running batches finish on the old lanes.
    void SetDevices(const std::vector<int>& devices);
    std::vector<int> Devices() const;           // resolved list
    std::vector<int> ConfiguredDevices() const; // as set (empty: default)
    // Smallest shard worth a second lane on the SAME device (items).
    void SetMinShard(size_t ecdsa, size_t equihash);
    // Smallest shard worth a device of its own (items); see PlanShards.
    void SetMinDeviceShard(size_t ecdsa, size_t equihash);
    // The plan a batch of n ECDSA (or Equihash) items would get on the current lanes.
    std::vector<VerifyShard> Plan(size_t n, bool equihash);

    // result[i] = 1 iff job i is valid (gpu::EcdsaVerifyBatch contract, packed arrays).
    std::vector<uint8_t> Ecdsa(const unsigned char* msg32, const unsigned char* sig64, const unsigned char* pub33,
                               size_t n);
    // The same batch with its inputs produced in place: fill(lo, hi, msg32, sig64, pub33, workers)
    // writes jobs [lo, hi) into a lane's pinned staging arrays (indexed from 0 = job lo), using
    // that lane's own fill workers.
    using EcdsaFillFn = std::function<void(size_t lo, size_t hi, unsigned char* msg32, unsigned char* sig64,
                                           unsigned char* pub33, WorkerPool& workers)>;
    std::vector<uint8_t> EcdsaFill(size_t n, const EcdsaFillFn& fill);
    // The same with DER signatures: the fill writes gpu::VerifyLane::DER_SLOT-byte slots
    // ([length][DER bytes]) where EcdsaFill takes 64-byte compact signatures; the device parses
    // them (lax rules) and low-S normalises.
    std::vector<uint8_t> EcdsaDerFill(size_t n, const EcdsaFillFn& fill);
    // Block headers [0, n): fill(lo, hi, in140, sols, lenok, workers) writes headers [lo, hi)
    // (gpu::VerifyLane::EquihashHeaders layout); the device builds the BLAKE2b states.
    using HeaderFillFn = std::function<void(size_t lo, size_t hi, uint8_t* in140, uint8_t* sols, uint8_t* lenok,
                                            WorkerPool& workers)>;
    std::vector<uint8_t> EquihashHeaders(unsigned N, unsigned K, size_t n, const HeaderFillFn& fill);
    // result[i] = 1 iff solution i is valid for state i.
    std::vector<uint8_t> Equihash(unsigned N, unsigned K, const std::vector<gpu::EhBaseState>& states,
                                  const std::vector<const std::vector<unsigned char>*>& sols);

    struct LaneStats {
        int device;
        int priority;
        uint64_t batches, items;
        uint64_t fillMicros, deviceMicros; // host fill vs device share of the lane's batches
        uint64_t ecdsaItems, equihashItems; // items by kind (signatures / header solutions)
    };
    std::vector<LaneStats> Stats() const;
    uint64_t ShardedBatches() const;
    // Stops the service threads (process shutdown; later calls restart them).
    void Shutdown();

private:
    GpuVerifyService() = default;
    struct Lane {
        int device = 0;
        std::unique_ptr<gpu::VerifyLane> gl; // created on the lane's own thread
        std::thread th;
        std::mutex m;
        std::condition_variable cv;
        std::deque<std::function<void()>> q;
        bool stop = false;
        std::string initError;
        std::atomic<int> priority{0};
        std::atomic<uint64_t> batches{0}, items{0};
        std::atomic<uint64_t> ecdsaItems{0}, equihashItems{0};
        std::atomic<uint64_t> fillMicros{0}, deviceMicros{0}; // the lane's host fill vs device time
        std::unique_ptr<WorkerPool> fill; // this lane's host-fill workers
    };
    static void LaneLoop(Lane* L);
    std::vector<std::shared_ptr<Lane>> AcquireLanes();
    // Runs fn(lane, lo, hi, workers) for the shards of [0, n) and waits; rethrows the first failure.
    void RunSharded(size_t n, bool equihash,
                    const std::function<void(gpu::VerifyLane&, size_t, size_t, WorkerPool&)>& fn);
    std::vector<uint8_t> EcdsaFillImpl(size_t n, bool der, const EcdsaFillFn& fill);

    mutable std::mutex m;
    std::vector<int> devices;
    std::vector<std::shared_ptr<Lane>> lanes;
    bool lanesStale = true;
    // smallest shard worth a second lane on one device (see AllDevices in gpuverify.cpp)
    size_t minShardEcdsa = 65536, minShardEquihash = 2048;
    // smallest shard worth a device of its own: the ECDSA floor is the batch at which the
    // verify kernel's fixed latency stops dominating (profiles/ecdsa_r5.md), the header floor a
    // few hundred headers (one workgroup per header, 0.2 ms per 2000)
    size_t minDevEcdsa = 4096, minDevEquihash = 256;
    uint64_t sharded = 0;
};

} // namespace bcp
