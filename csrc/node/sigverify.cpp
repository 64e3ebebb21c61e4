#include "node/sigverify.h"
#include "kernels/gpu_api.h"
#include "node/gpuverify.h"
#include "keys/key.h"
#include "secp256k1/secp256k1.h"

#include <atomic>
#include <cstring>
#include <future>

namespace bcp {

SignatureCache::SignatureCache() {
    GetRandBytes(nonce.begin(), 32);
    set.setup_bytes((size_t)DEFAULT_MAX_SIG_CACHE_SIZE << 20);
}

uint256 SignatureCache::Entry(const uint256& sighash, const unsigned char* sig, size_t sigLen,
                              const unsigned char* pubkey, size_t pubLen) const {
    CSHA256 h;
    h.Write(nonce.begin(), 32).Write(sighash.begin(), 32).Write(pubkey, pubLen).Write(sig, sigLen);
    uint256 r;
    h.Finalize(r.begin());
    return r;
}
SignatureCache& GetSignatureCache() {
    static SignatureCache c;
    return c;
}
size_t InitSignatureCache(int64_t mib) {
    mib = std::min(std::max<int64_t>(0, mib), MAX_MAX_SIG_CACHE_SIZE);
    const size_t n = GetSignatureCache().SetupBytes((size_t)mib << 20);
    LogPrintf("Using %zu MiB out of %zu requested for signature cache, able to store %zu elements\n",
              (n * sizeof(uint256)) >> 20, (size_t)mib, n);
    return n;
}

static std::atomic<size_t> g_gpuThreshold{DEFAULT_GPU_SIG_THRESHOLD};
void SetGpuSigThreshold(size_t n) { g_gpuThreshold = n; }
size_t GetGpuSigThreshold() { return g_gpuThreshold.load(); }

// Device failures (allocation, launch, fault) never decide a block's validity: the batch
// is re-verified on the CPU. After MAX_GPU_SIG_FAILURES consecutive failures the GPU
// path is switched off for the rest of the process.
static std::atomic<int> g_gpuFailures{0};
static std::atomic<bool> g_gpuDisabled{false};
void ResetGpuSigFailures() {
    g_gpuFailures = 0;
    g_gpuDisabled = false;
}
bool GpuSigPathDisabled() { return g_gpuDisabled.load(); }
bool GpuBatchesExpected(bool useGpu) {
    return useGpu && !g_gpuDisabled.load() && (GpuFaultInjection() || gpu::GpuAvailable());
}

static std::mutex g_statsMutex;
static SigVerifyStats g_stats;
SigVerifyStats GetSigVerifyStats() {
    std::lock_guard<std::mutex> l(g_statsMutex);
    return g_stats;
}

bool CachingTransactionSignatureChecker::VerifySignature(const std::vector<unsigned char>& sig,
                                                         const std::vector<unsigned char>& pubkey,
                                                         const uint256& sighash) const {
    SignatureCache& cache = GetSignatureCache();
    const uint256 e = cache.Entry(sighash, sig, pubkey);
    if (cache.Get(e, !store)) return true;
    if (!TransactionSignatureChecker::VerifySignature(sig, pubkey, sighash)) return false;
    if (store) cache.Set(e);
    return true;
}

// Host half of one job on the device-DER path: the raw DER bytes into their slot (the device
// parses and normalises them) and the key in compressed form. A key that does not parse keeps
// the device input well-formed; false masks its result.
static bool PrepDerAndKey(const DeferredSigCheck& c, unsigned char* slot, unsigned char* pub33) {
    const size_t len = c.sig.size(); // <= 72 (InlineBytes<72>)
    slot[0] = (unsigned char)len;
    memcpy(slot + 1, c.sig.data(), len);
    const auto& pk = c.pubkey;
    if (pk.size() == 33 && (pk[0] == 2 || pk[0] == 3)) {
        memcpy(pub33, pk.data(), 33);
        return true;
    }
    secp::Ge q;
    if (secp::pubkey_parse(q, pk.data(), pk.size())) {
        std::vector<unsigned char> comp = secp::pubkey_serialize(q, true);
        memcpy(pub33, comp.data(), 33);
        return true;
    }
    memset(pub33, 0, 33);
    pub33[0] = 2;
    return false;
}

std::vector<uint8_t> GpuVerifyDeferred(const std::vector<const DeferredSigCheck*>& checks) {
    // host: copy the digest, the DER bytes and the key (converted to compressed form when it is
    // not) straight into the verify lane's pinned staging buffer; device: DER parse + low-S,
    // scalar prep, decompression + ecmult
    const size_t n = checks.size();
    std::vector<uint8_t> hostOk(n, 1);
    if (GpuFaultInjection()) throw std::runtime_error("injected GPU signature-verify fault");
    // each lane's shard is filled by that lane's own workers, concurrently with the other lanes
    auto fill = [&](size_t lo, size_t hi, unsigned char* msg, unsigned char* sig, unsigned char* pub,
                    WorkerPool& workers) {
        workers.ParallelFor(
            hi - lo,
            [&](size_t k) {
                const DeferredSigCheck& c = *checks[lo + k];
                memcpy(&msg[k * 32], c.sighash.begin(), 32);
                if (!PrepDerAndKey(c, &sig[k * gpu::VerifyLane::DER_SLOT], &pub[k * 33])) hostOk[lo + k] = 0;
            },
            256);
    };
    // sharded across the validation GPUs by the verify service (one high-priority lane each)
    std::vector<uint8_t> res = GpuVerifyService::Instance().EcdsaDerFill(n, fill);
    for (size_t j = 0; j < n; j++) res[j] &= hostOk[j];
    return res;
}

bool BatchVerifySignatures(std::vector<DeferredSigCheck>& checks, WorkerPool* pool, bool useGpu, bool cacheStore,
                           bool cacheErase) {
    static const std::vector<DeferredMultisig> none;
    return BatchVerifySignatures(checks, none, pool, useGpu, cacheStore, cacheErase);
}

bool BatchVerifySignatures(std::vector<DeferredSigCheck>& checks, const std::vector<DeferredMultisig>& groups,
                           WorkerPool* pool, bool useGpu, bool cacheStore, bool cacheErase) {
    std::vector<const DeferredSigCheck*> ptrs(checks.size());
    for (size_t i = 0; i < checks.size(); i++) ptrs[i] = &checks[i];
    return BatchVerifySignatures(ptrs, groups, pool, useGpu, cacheStore, cacheErase);
}

bool BatchVerifySignatures(const std::vector<const DeferredSigCheck*>& checks,
                           const std::vector<DeferredMultisig>& groups, WorkerPool* pool, bool useGpu,
                           bool cacheStore, bool cacheErase) {
    if (checks.empty()) return groups.empty();
    // speculative pairs of deferred multisig groups: their individual results are kept, and a false
    // one does not fail the batch
    std::vector<uint8_t> spec(checks.size(), 0), res(checks.size(), 0);
    for (const DeferredMultisig& g : groups) {
        if ((size_t)g.first + g.Pairs() > checks.size()) return false; // malformed group: never valid
        std::fill(spec.begin() + g.first, spec.begin() + g.first + g.Pairs(), 1);
    }
    SignatureCache& cache = GetSignatureCache();
    std::vector<uint256> entries(checks.size());
    std::vector<uint8_t> hit(checks.size());
    std::vector<size_t> todo;
    todo.reserve(checks.size());
    uint64_t hits = 0;
    // cache keys are one SHA-256 each: on the pool, in chunks whose lookups share one lock
    const size_t PROBE_CHUNK = 256;
    // nothing was ever stored and nothing will be: every probe would miss (initial sync)
    const bool skipProbes = !cacheStore && !cache.MayHold();
    auto probe = [&](size_t chunk) {
        if (skipProbes) return;
        const size_t lo = chunk * PROBE_CHUNK, hi = std::min(checks.size(), lo + PROBE_CHUNK);
        for (size_t i = lo; i < hi; i++) {
            const DeferredSigCheck& c = *checks[i];
            entries[i] = cache.Entry(c.sighash, c.sig.data(), c.sig.size(), c.pubkey.data(), c.pubkey.size());
        }
        cache.GetMany(&entries[lo], hi - lo, cacheErase, &hit[lo]);
    };
    const size_t nChunks = (checks.size() + PROBE_CHUNK - 1) / PROBE_CHUNK;
    // A cold cache (initial sync, a block nobody relayed first): when the first chunk's probes
    // mostly miss, the whole batch goes to the GPU right away and the remaining probes run on the
    // CPU meanwhile; a hit then only saves the cache insert. A warm cache (a synced node, whose
    // mempool already verified most of the block) keeps probe-first, so hits never wait for the
    // GPU. Either way res[i] = hit or verified.
    bool gpuFailedEarly = false; // the overlapped GPU batch below failed: the rest stays on the CPU
    const bool gpuEligible = useGpu && !g_gpuDisabled.load() && checks.size() >= g_gpuThreshold.load() &&
                             (GpuFaultInjection() || gpu::GpuAvailable());
    if (gpuEligible && nChunks > 1) {
        probe(0);
        size_t sampleHits = 0;
        for (size_t i = 0; i < PROBE_CHUNK; i++) sampleHits += hit[i];
        if (sampleHits * 2 < PROBE_CHUNK) {
            auto gpuRun = std::async(std::launch::async, [&checks] { return GpuVerifyDeferred(checks); });
            const int64_t t0 = GetTimeMicros();
            if (skipProbes) {
                // nothing to probe: the pool stays free for other work while the GPU runs
            } else if (pool) {
                pool->ParallelFor(nChunks - 1, [&](size_t k) { probe(k + 1); }, 1);
            } else {
                for (size_t k = 1; k < nChunks; k++) probe(k);
            }
            std::vector<uint8_t> r;
            bool gpuOk = true;
            try {
                r = gpuRun.get();
                g_gpuFailures = 0;
            } catch (const std::exception& e) {
                gpuOk = false;
                const int fails = ++g_gpuFailures;
                LogPrintf("GPU signature verification failed (%s); re-verifying on the CPU\n", e.what());
                if (fails >= MAX_GPU_SIG_FAILURES && !g_gpuDisabled.exchange(true))
                    LogPrintf("GPU signature verification disabled after %d consecutive failures\n", fails);
                std::lock_guard<std::mutex> l(g_statsMutex);
                g_stats.gpu_failures++;
            }
            if (gpuOk) {
                bool ok = true;
                for (size_t i = 0; i < checks.size(); i++) {
                    if (hit[i]) {
                        hits++;
                        res[i] = 1;
                    } else {
                        res[i] = r[i];
                        if (!r[i]) {
                            if (!spec[i]) ok = false;
                        } else if (cacheStore) {
                            cache.Set(entries[i]);
                        }
                    }
                }
                if (ok)
                    for (const DeferredMultisig& g : groups)
                        if (!EvalDeferredMultisig(g, &res[g.first])) {
                            ok = false;
                            break;
                        }
                std::lock_guard<std::mutex> l(g_statsMutex);
                g_stats.gpu_batches++;
                g_stats.gpu_sigs += checks.size();
                g_stats.gpu_ms += (GetTimeMicros() - t0) / 1000.0;
                g_stats.cache_hits += hits;
                g_stats.multisig_groups += groups.size();
                return ok;
            }
            // the GPU failed: the probes are complete; the CPU path below verifies the misses
            gpuFailedEarly = true;
        } else if (pool) {
            pool->ParallelFor(nChunks - 1, [&](size_t k) { probe(k + 1); }, 1);
        } else {
            for (size_t k = 1; k < nChunks; k++) probe(k);
        }
    } else if (pool && nChunks > 1) {
        pool->ParallelFor(nChunks, probe, 1);
    } else {
        for (size_t k = 0; k < nChunks; k++) probe(k);
    }
    for (size_t i = 0; i < checks.size(); i++) {
        if (hit[i]) {
            hits++;
            res[i] = 1;
        } else {
            todo.push_back(i);
        }
    }
    bool ok = true;
    const size_t n = todo.size();
    if (n > 0) {
        bool gpu = !gpuFailedEarly && useGpu && !g_gpuDisabled.load() && n >= g_gpuThreshold.load() &&
                   (GpuFaultInjection() || gpu::GpuAvailable());
        const int64_t t0 = GetTimeMicros();
        if (gpu) {
            std::vector<const DeferredSigCheck*> ptrs(n);
            for (size_t j = 0; j < n; j++) ptrs[j] = checks[todo[j]];
            std::vector<uint8_t> r;
            try {
                r = GpuVerifyDeferred(ptrs);
                g_gpuFailures = 0;
            } catch (const std::exception& e) {
                const int fails = ++g_gpuFailures;
                LogPrintf("GPU signature verification failed (%s); re-verifying %zu signatures on the CPU\n",
                          e.what(), n);
                if (fails >= MAX_GPU_SIG_FAILURES && !g_gpuDisabled.exchange(true))
                    LogPrintf("GPU signature verification disabled after %d consecutive failures\n", fails);
                std::lock_guard<std::mutex> l(g_statsMutex);
                g_stats.gpu_failures++;
                gpu = false;
            }
            if (gpu) {
                for (size_t j = 0; j < n; j++) {
                    res[todo[j]] = r[j];
                    if (!r[j]) {
                        if (!spec[todo[j]]) ok = false;
                    } else if (cacheStore) {
                        cache.Set(entries[todo[j]]);
                    }
                }
                std::lock_guard<std::mutex> l(g_statsMutex);
                g_stats.gpu_batches++;
                g_stats.gpu_sigs += n;
                g_stats.gpu_ms += (GetTimeMicros() - t0) / 1000.0;
            }
        }
        if (!gpu) {
            std::atomic<bool> allOk{true};
            auto work = [&](size_t j) {
                if (!allOk.load(std::memory_order_relaxed)) return;
                const size_t i = todo[j];
                const DeferredSigCheck& c = *checks[i];
                res[i] = secp::VerifySignature(c.pubkey.data(), c.pubkey.size(), c.sig.data(), c.sig.size(),
                                               c.sighash.begin());
                if (!res[i]) {
                    if (!spec[i]) allOk = false;
                } else if (cacheStore) {
                    cache.Set(entries[i]);
                }
            };
            if (pool) pool->ParallelFor(n, work, 8);
            else for (size_t j = 0; j < n; j++) work(j);
            ok = allOk.load();
            std::lock_guard<std::mutex> l(g_statsMutex);
            g_stats.cpu_sigs += n;
            g_stats.cpu_ms += (GetTimeMicros() - t0) / 1000.0;
        }
    }
    if (ok)
        for (const DeferredMultisig& g : groups)
            if (!EvalDeferredMultisig(g, &res[g.first])) {
                ok = false;
                break;
            }
    std::lock_guard<std::mutex> l(g_statsMutex);
    g_stats.cache_hits += hits;
    g_stats.multisig_groups += groups.size();
    return ok;
}

} // namespace bcp
