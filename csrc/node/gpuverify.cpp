#include "node/gpuverify.h"

#include "util/util.h"

#include <algorithm>
#include <atomic>
#include <exception>
#include <cstdlib>
#include <stdexcept>

namespace bcp {

std::vector<VerifyShard> PlanShards(size_t n, const std::vector<int>& laneDevices, size_t minPerDevice,
                                    size_t minPerLane) {
    std::vector<VerifyShard> plan;
    if (n == 0 || laneDevices.empty()) return plan;
    minPerDevice = std::max<size_t>(1, minPerDevice);
    minPerLane = std::max<size_t>(1, minPerLane);
    std::vector<int> devs;                  // distinct devices, first-listed order
    std::vector<std::vector<size_t>> lanes; // lanes of each
    for (size_t i = 0; i < laneDevices.size(); i++) {
        const auto it = std::find(devs.begin(), devs.end(), laneDevices[i]);
        if (it == devs.end()) {
            devs.push_back(laneDevices[i]);
            lanes.push_back({i});
        } else {
            lanes[it - devs.begin()].push_back(i);
        }
    }
    const size_t k = std::max<size_t>(1, std::min(devs.size(), n / minPerDevice));
    size_t lo = 0;
    for (size_t d = 0; d < k; d++) {
        const size_t share = n / k + (d < n % k ? 1 : 0);
        const size_t nl = std::max<size_t>(1, std::min(lanes[d].size(), share / minPerLane));
        for (size_t l = 0; l < nl; l++) {
            const size_t part = share / nl + (l < share % nl ? 1 : 0);
            plan.push_back(VerifyShard{lanes[d][l], lo, lo + part});
            lo += part;
        }
    }
    return plan;
}

GpuVerifyService& GpuVerifyService::Instance() {
    static GpuVerifyService s;
    return s;
}

GpuVerifyService::~GpuVerifyService() { Shutdown(); }

void GpuVerifyService::Shutdown() {
    std::vector<std::shared_ptr<Lane>> old;
    {
        std::lock_guard<std::mutex> l(m);
        old.swap(lanes);
        lanesStale = true;
    }
    for (auto& L : old) {
        {
            std::lock_guard<std::mutex> l(L->m);
            L->stop = true;
        }
        L->cv.notify_all();
        if (L->th.joinable()) L->th.join();
    }
}

void GpuVerifyService::SetDevices(const std::vector<int>& devs) {
    std::lock_guard<std::mutex> l(m);
    devices = devs;
    lanesStale = true;
}

// Default: every visible device, two lanes each (the built-in miner runs only on demand, and
// its streams share a device at a lower priority than validation's), listed device by device
// round-robin ([0, 1, .., n-1, 0, 1, ..]). PlanShards spreads a batch over distinct devices
// first; a second lane on one device takes a shard only at >= minShardEcdsa signatures: two
// kernels of one batch on the same device do not overlap (each waits out the verify latency),
// so an 8 MB block's 42k-signature batch took 3.3 ms device time whole and 7.5 ms in two shards
// on one GPU; only the 199k worst case gains from a second lane there (profiles/connect_r4.md).
// A process that is one rank of a multi-process job (WORLD_SIZE > 1 with LOCAL_RANK set, one
// process per GPU) keeps to its own device instead of placing streams on its neighbours'.
static std::vector<int> AllDevices() {
    std::vector<int> d;
    if (!gpu::GpuAvailable()) return d;
    const int n = gpu::DeviceCount();
    const char* ws = getenv("WORLD_SIZE");
    const char* lr = getenv("LOCAL_RANK");
    if (ws && lr && atoi(ws) > 1 && n > 0) {
        const int own = atoi(lr) % n;
        return {own, own};
    }
    for (int rep = 0; rep < 2; rep++)
        for (int i = 0; i < n; i++) d.push_back(i);
    return d;
}

std::vector<int> GpuVerifyService::Devices() const {
    std::lock_guard<std::mutex> l(m);
    if (!devices.empty()) return devices;
    return AllDevices();
}

std::vector<int> GpuVerifyService::ConfiguredDevices() const {
    std::lock_guard<std::mutex> l(m);
    return devices;
}

void GpuVerifyService::SetMinShard(size_t ecdsa, size_t equihash) {
    std::lock_guard<std::mutex> l(m);
    minShardEcdsa = std::max<size_t>(1, ecdsa);
    minShardEquihash = std::max<size_t>(1, equihash);
}

void GpuVerifyService::SetMinDeviceShard(size_t ecdsa, size_t equihash) {
    std::lock_guard<std::mutex> l(m);
    minDevEcdsa = std::max<size_t>(1, ecdsa);
    minDevEquihash = std::max<size_t>(1, equihash);
}

std::vector<VerifyShard> GpuVerifyService::Plan(size_t n, bool equihash) {
    std::vector<int> devs;
    {
        std::lock_guard<std::mutex> l(m);
        if (!lanesStale) {
            for (const auto& L : lanes) devs.push_back(L->device);
        } else {
            devs = devices.empty() ? AllDevices() : devices;
        }
        return PlanShards(n, devs, equihash ? minDevEquihash : minDevEcdsa,
                          equihash ? minShardEquihash : minShardEcdsa);
    }
}

void GpuVerifyService::LaneLoop(Lane* L) {
    RenameThread(("bcp-gpuverify" + std::to_string(L->device)).c_str());
    try {
        L->gl.reset(new gpu::VerifyLane(L->device, /*highPriority=*/true));
        L->priority = L->gl->Priority();
    } catch (const std::exception& e) {
        L->initError = e.what();
    }
    for (;;) {
        std::function<void()> task;
        {
            std::unique_lock<std::mutex> l(L->m);
            L->cv.wait(l, [&] { return L->stop || !L->q.empty(); });
            if (L->q.empty()) break; // stop requested and nothing queued
            task = std::move(L->q.front());
            L->q.pop_front();
        }
        task(); // tasks check L->gl / initError themselves (see RunSharded)
    }
    L->gl.reset();
}

std::vector<std::shared_ptr<GpuVerifyService::Lane>> GpuVerifyService::AcquireLanes() {
    std::vector<std::shared_ptr<Lane>> retire;
    std::vector<std::shared_ptr<Lane>> cur;
    {
        std::lock_guard<std::mutex> l(m);
        if (lanesStale) {
            std::vector<int> devs = devices;
            if (devs.empty()) devs = AllDevices();
            retire.swap(lanes);
            // host-fill workers: the cores split between the lanes, at most 16 per lane (a fill is
            // a few hundred microseconds: waking more threads than that costs more than they
            // save). WorkerPool(k) has k participants: k - 1 threads plus the lane's own thread.
            const int perLane = std::min(16, std::max(1, (GetNumCores() - 1) / std::max<int>(1, (int)devs.size())));
            for (int d : devs) {
                auto L = std::make_shared<Lane>();
                L->device = d;
                L->fill.reset(new WorkerPool(perLane));
                L->th = std::thread(LaneLoop, L.get());
                lanes.push_back(L);
            }
            lanesStale = false;
        }
        cur = lanes;
    }
    for (auto& L : retire) { // old lanes finish what they hold, then exit
        {
            std::lock_guard<std::mutex> l(L->m);
            L->stop = true;
        }
        L->cv.notify_all();
        if (L->th.joinable()) L->th.join();
    }
    return cur;
}

void GpuVerifyService::RunSharded(size_t n, bool equihash,
                                  const std::function<void(gpu::VerifyLane&, size_t, size_t, WorkerPool&)>& fn) {
    std::vector<std::shared_ptr<Lane>> ls = AcquireLanes();
    if (ls.empty()) throw std::runtime_error("GpuVerifyService: no validation GPU");
    std::vector<int> laneDev;
    for (const auto& L : ls) laneDev.push_back(L->device);
    size_t minDev, minLane;
    {
        std::lock_guard<std::mutex> l(m);
        minDev = equihash ? minDevEquihash : minDevEcdsa;
        minLane = equihash ? minShardEquihash : minShardEcdsa;
    }
    const std::vector<VerifyShard> plan = PlanShards(n, laneDev, minDev, minLane);
    const size_t shards = plan.size();
    struct Latch {
        std::mutex m;
        std::condition_variable cv;
        size_t left;
        std::exception_ptr err;
    } latch;
    latch.left = shards;
    if (shards > 1) {
        std::lock_guard<std::mutex> l(m);
        sharded++;
    }
    for (size_t s = 0; s < shards; s++) {
        const size_t lo = plan[s].lo, hi = plan[s].hi;
        Lane* L = ls[plan[s].lane].get();
        auto task = [&fn, &latch, L, lo, hi, equihash]() {
            std::exception_ptr e;
            try {
                if (!L->gl) throw std::runtime_error("GPU verify lane on device " + std::to_string(L->device) +
                                                     " unavailable: " + L->initError);
                fn(*L->gl, lo, hi, *L->fill);
                L->batches++;
                L->items += hi - lo;
                (equihash ? L->equihashItems : L->ecdsaItems) += hi - lo;
                L->fillMicros = L->gl->FillMicros(); // published for Stats() (this is the lane's thread)
                L->deviceMicros = L->gl->DeviceMicros();
            } catch (...) {
                e = std::current_exception();
            }
            std::lock_guard<std::mutex> l(latch.m);
            if (e && !latch.err) latch.err = e;
            if (--latch.left == 0) latch.cv.notify_all();
        };
        bool queued = false;
        {
            std::lock_guard<std::mutex> l(L->m);
            if (!L->stop) { // a lane retired by a concurrent SetDevices takes no new work
                L->q.push_back(task);
                queued = true;
            }
        }
        if (queued) {
            L->cv.notify_one();
        } else {
            std::lock_guard<std::mutex> l(latch.m);
            if (!latch.err) latch.err = std::make_exception_ptr(std::runtime_error("GPU verify lane retired"));
            --latch.left;
        }
    }
    std::unique_lock<std::mutex> l(latch.m);
    latch.cv.wait(l, [&] { return latch.left == 0; });
    if (latch.err) std::rethrow_exception(latch.err);
}

std::vector<uint8_t> GpuVerifyService::Ecdsa(const unsigned char* msg32, const unsigned char* sig64,
                                             const unsigned char* pub33, size_t n) {
    std::vector<uint8_t> out(n, 0);
    if (n == 0) return out;
    RunSharded(n, false, [&](gpu::VerifyLane& lane, size_t lo, size_t hi, WorkerPool&) {
        lane.Ecdsa(msg32 + lo * 32, sig64 + lo * 64, pub33 + lo * 33, hi - lo, out.data() + lo);
    });
    return out;
}

std::vector<uint8_t> GpuVerifyService::EcdsaFillImpl(size_t n, bool der, const EcdsaFillFn& fill) {
    std::vector<uint8_t> out(n, 0);
    if (n == 0) return out;
    RunSharded(n, false, [&](gpu::VerifyLane& lane, size_t lo, size_t hi, WorkerPool& workers) {
        auto f = [&](unsigned char* msg, unsigned char* sig, unsigned char* pub) { fill(lo, hi, msg, sig, pub, workers); };
        if (der) lane.EcdsaDerFill(hi - lo, f, out.data() + lo);
        else lane.EcdsaFill(hi - lo, f, out.data() + lo);
    });
    return out;
}

std::vector<uint8_t> GpuVerifyService::EcdsaFill(size_t n, const EcdsaFillFn& fill) { return EcdsaFillImpl(n, false, fill); }

std::vector<uint8_t> GpuVerifyService::EcdsaDerFill(size_t n, const EcdsaFillFn& fill) { return EcdsaFillImpl(n, true, fill); }

std::vector<uint8_t> GpuVerifyService::EquihashHeaders(unsigned N, unsigned K, size_t n, const HeaderFillFn& fill) {
    std::vector<uint8_t> out(n, 0);
    if (n == 0) return out;
    RunSharded(n, true, [&](gpu::VerifyLane& lane, size_t lo, size_t hi, WorkerPool& workers) {
        lane.EquihashHeaders(
            N, K, hi - lo, [&](uint8_t* in, uint8_t* sols, uint8_t* lenok) { fill(lo, hi, in, sols, lenok, workers); },
            out.data() + lo);
    });
    return out;
}

std::vector<uint8_t> GpuVerifyService::Equihash(unsigned N, unsigned K, const std::vector<gpu::EhBaseState>& states,
                                                const std::vector<const std::vector<unsigned char>*>& sols) {
    if (states.size() != sols.size()) throw std::invalid_argument("GpuVerifyService::Equihash: sizes");
    const size_t n = states.size();
    std::vector<uint8_t> out(n, 0);
    if (n == 0) return out;
    RunSharded(n, true, [&](gpu::VerifyLane& lane, size_t lo, size_t hi, WorkerPool&) {
        lane.Equihash(N, K, states.data() + lo, sols.data() + lo, hi - lo, out.data() + lo);
    });
    return out;
}

uint64_t GpuVerifyService::ShardedBatches() const {
    std::lock_guard<std::mutex> l(m);
    return sharded;
}

std::vector<GpuVerifyService::LaneStats> GpuVerifyService::Stats() const {
    std::vector<LaneStats> out;
    std::lock_guard<std::mutex> l(m);
    for (const auto& L : lanes) {
        out.push_back(LaneStats{L->device, L->priority.load(), L->batches.load(), L->items.load(),
                                L->fillMicros.load(), L->deviceMicros.load(), L->ecdsaItems.load(),
                                L->equihashItems.load()});
    }
    return out;
}

} // namespace bcp
