// Signature cache and batched ECDSA verification (CPU pool or MI355X).
// Parity: reference src/script/sigcache.{h,cpp} (salted cache of valid (sighash,
// pubkey, sig) triples, -maxsigcachesize, erase-on-block-use) and src/checkqueue.h
// (CCheckQueue fan-out of CScriptCheck across -par threads). Here script evaluation
// runs on the CPU pool and the deferred ECDSA checks (interpreter.h) are verified in
// one batch: on the GPU when available and the batch is large enough, else on the pool.
#pragma once
#include <atomic>
#include "script/interpreter.h"
#include "util/cuckoocache.h"
#include "util/util.h"

#include <unordered_set>

namespace bcp {

static const unsigned DEFAULT_MAX_SIG_CACHE_SIZE = 32;    // MiB (reference sigcache.h:16)
static const int64_t MAX_MAX_SIG_CACHE_SIZE = 16384;        // MiB
static const unsigned DEFAULT_MAX_SCRIPT_CACHE_SIZE = 32; // MiB (reference scriptcache.h:17)
static const int64_t MAX_MAX_SCRIPT_CACHE_SIZE = 16384;

// Salted cuckoo set of verified (sighash, pubkey, sig) triples.
class SignatureCache {
public:
    SignatureCache();
    bool Get(const uint256& entry, bool erase) const { return set.contains(entry, erase); }
    void Set(const uint256& entry) {
        if (!everSet.load(std::memory_order_relaxed)) everSet.store(true, std::memory_order_relaxed);
        set.insert(entry);
    }
    // false while nothing was ever stored (a node in initial sync, whose blocks' signatures were
    // never seen in its mempool): a probe could only miss, so a batch skips the probes
    bool MayHold() const { return everSet.load(std::memory_order_relaxed); }
    void GetMany(const uint256* entries, size_t n, bool erase, uint8_t* hit) const {
        set.contains_many(entries, n, erase, hit);
    }
    uint256 Entry(const uint256& sighash, const unsigned char* sig, size_t sigLen, const unsigned char* pubkey,
                  size_t pubLen) const;
    uint256 Entry(const uint256& sighash, const std::vector<unsigned char>& sig,
                  const std::vector<unsigned char>& pubkey) const {
        return Entry(sighash, sig.data(), sig.size(), pubkey.data(), pubkey.size());
    }
    size_t SetupBytes(size_t bytes) { return set.setup_bytes(bytes); }
    size_t Capacity() const { return set.capacity(); }
    size_t Size() const { return set.count_live(); }

private:
    uint256 nonce;
    SharedCuckooSet set;
    std::atomic<bool> everSet{false};
};
SignatureCache& GetSignatureCache();
// -maxsigcachesize / -maxscriptcachesize (MiB); returns element capacities.
size_t InitSignatureCache(int64_t mib);

struct SigVerifyStats {
    uint64_t gpu_batches = 0, gpu_sigs = 0, cpu_sigs = 0, cache_hits = 0, gpu_failures = 0;
    uint64_t multisig_groups = 0; // CHECKMULTISIGs verified through the batch (speculative pairs)
    double gpu_ms = 0, cpu_ms = 0;
};

// Smallest batch sent to the GPU (-gpusigthreshold). Below it the CPU pool is faster:
// profiles/ecdsa_r5.md measures the crossover on MI355X. With the fused latency kernel a batch
// of up to 8192 signatures takes 0.86-0.98 ms end to end; the 16-thread pool's best rate
// (139k sig/s) needs 0.92 ms for 128. (It was 512 with the 2.6 ms split kernels,
// profiles/ecdsa_r2_regular.md, and 1024 before that.)
static const size_t DEFAULT_GPU_SIG_THRESHOLD = 128;
// Consecutive device failures after which the GPU signature path is turned off.
static const int MAX_GPU_SIG_FAILURES = 3;

// Verify all checks; returns true iff every one is valid. cacheStore: remember
// successes (mempool acceptance); block validation erases consumed entries.
bool BatchVerifySignatures(std::vector<DeferredSigCheck>& checks, WorkerPool* pool, bool useGpu, bool cacheStore,
                           bool cacheErase);
// Same, with deferred CHECKMULTISIG groups: their pair checks are speculative (a false pair is
// legal), and each group must pass its replayed greedy match instead.
bool BatchVerifySignatures(std::vector<DeferredSigCheck>& checks, const std::vector<DeferredMultisig>& groups,
                           WorkerPool* pool, bool useGpu, bool cacheStore, bool cacheErase);
// Same, over checks that stay where they were produced (the block path's per-job sinks): no copy
// into one array first.
bool BatchVerifySignatures(const std::vector<const DeferredSigCheck*>& checks,
                           const std::vector<DeferredMultisig>& groups, WorkerPool* pool, bool useGpu,
                           bool cacheStore, bool cacheErase);
// Device verification of the given checks (no cache); result[i] = 1 iff valid.
std::vector<uint8_t> GpuVerifyDeferred(const std::vector<const DeferredSigCheck*>& checks);
void SetGpuSigThreshold(size_t n);   // minimum batch size for the GPU path
size_t GetGpuSigThreshold();
void ResetGpuSigFailures();
bool GpuSigPathDisabled();
// Whether large batches would go to the GPU: CHECKMULTISIG is deferred speculatively (more pairs
// than the eager match checks) only then; a CPU-only node keeps the eager match on its workers.
bool GpuBatchesExpected(bool useGpu);
SigVerifyStats GetSigVerifyStats();

// TransactionSignatureChecker that consults/updates the signature cache.
class CachingTransactionSignatureChecker : public TransactionSignatureChecker {
public:
    CachingTransactionSignatureChecker(const CTransaction* tx, unsigned nIn, Amount amount, bool store,
                                       const PrecomputedTransactionData* txdata)
        : TransactionSignatureChecker(tx, nIn, amount, txdata), store(store) {}

protected:
    bool VerifySignature(const std::vector<unsigned char>& sig, const std::vector<unsigned char>& pubkey,
                         const uint256& sighash) const override;

private:
    bool store;
};

} // namespace bcp
