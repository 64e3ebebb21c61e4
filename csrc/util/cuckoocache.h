// Fixed-memory set of already-salted 256-bit hashes, used by the signature cache and
// the script-execution cache.
// Parity: reference src/cuckoocache.h:156 (CuckooCache::cache: bounded-memory cuckoo
// table, 8 candidate slots per element, lock-free erase via garbage flags, generation
// aging so recently inserted entries survive eviction) and its users
// src/script/sigcache.cpp:70 / src/script/scriptcache.cpp:19 (-maxsigcachesize /
// -maxscriptcachesize in MiB).
//
// Design:
//   * Keys are uniformly random (salted SHA256 outputs), so the 8 slot indices come
//     straight from the key's eight 32-bit words with a multiply-shift range reduction;
//     no extra hashing.
//   * Per-slot state lives in one byte (occupied / collectable / current generation).
//     Lookups and erases only touch that byte with relaxed atomics, so many readers (block
//     validation worker threads) can probe and erase under a shared lock while inserts
//     take the exclusive lock (SharedCuckooSet below).
//   * Insert: first free/dead slot among the 8 wins; otherwise a bounded cuckoo walk
//     (depth ~ log2(size)) displaces entries, preferring previous-generation victims.
//     When the current generation's un-erased entries reach ~45% of the table it becomes
//     the old generation and the previous old generation turns collectable (still
//     answering lookups until overwritten) - recent entries, the ones blocks are about
//     to consume, are never the first to go.
#pragma once
#include "primitives/uint256.h"

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <vector>

namespace bcp {

class CuckooHashSet {
public:
    static constexpr int WAYS = 8;
    // OCC: slot holds a key. COLLECT: key may be overwritten (erased or aged out) but
    // still answers lookups until it is. GEN: inserted in the current generation.
    enum : uint8_t { OCC = 1, COLLECT = 2, GEN = 4 };

    CuckooHashSet() { setup(2); }

    // Size the table to `bytes` of key storage; returns the element capacity (>= 2).
    size_t setup_bytes(size_t bytes) { return setup(std::max<size_t>(2, bytes / sizeof(uint256))); }

    size_t setup(size_t n) {
        n = std::max<size_t>(2, n);
        keys.assign(n, uint256());
        state.reset(new std::atomic<uint8_t>[n]);
        for (size_t i = 0; i < n; ++i) state[i].store(0, std::memory_order_relaxed);
        size = n;
        depth = 1;
        while ((size_t(1) << depth) < n) ++depth;
        genLimit = std::max<size_t>(1, (n * 45) / 100);
        untilCheck = genLimit;
        return n;
    }

    size_t capacity() const { return size; }

    // True iff `k` is present. erase=true marks a hit collectable (lock-free; safe
    // concurrently with other contains() calls).
    bool contains(const uint256& k, bool erase) const {
        uint32_t idx[WAYS];
        slots(k, idx);
        for (int w = 0; w < WAYS; ++w) {
            const uint32_t i = idx[w];
            if ((state[i].load(std::memory_order_relaxed) & OCC) && keys[i] == k) {
                if (erase) state[i].fetch_or(COLLECT, std::memory_order_relaxed);
                return true;
            }
        }
        return false;
    }

    // Insert (caller holds exclusive access). A key already present is refreshed into
    // the current generation rather than stored twice.
    void insert(const uint256& key) {
        uint256 k = key;
        uint32_t idx[WAYS];
        slots(k, idx);
        for (int w = 0; w < WAYS; ++w) {
            const uint32_t i = idx[w];
            if ((state[i].load(std::memory_order_relaxed) & OCC) && keys[i] == k) {
                const uint8_t st = state[i].load(std::memory_order_relaxed);
                state[i].store((uint8_t)(OCC | GEN), std::memory_order_relaxed);
                if ((st & (GEN | COLLECT)) != GEN) tick();
                return;
            }
        }
        uint8_t kgen = GEN;
        for (unsigned step = 0; step <= depth; ++step) {
            for (int w = 0; w < WAYS; ++w) { // empty or collectable slot
                const uint32_t i = idx[w];
                const uint8_t st = state[i].load(std::memory_order_relaxed);
                if (!(st & OCC) || (st & COLLECT)) {
                    place(i, k, kgen);
                    return;
                }
            }
            // displace: prefer a previous-generation entry, else rotate through the ways
            int victim = -1;
            for (int w = 0; w < WAYS && victim < 0; ++w)
                if (!(state[idx[w]].load(std::memory_order_relaxed) & GEN)) victim = w;
            if (victim < 0) victim = (int)(rot++ % WAYS);
            const uint32_t vi = idx[victim];
            const uint8_t vgen = state[vi].load(std::memory_order_relaxed) & GEN;
            const uint256 evicted = keys[vi];
            place(vi, k, kgen);
            if (step == depth) return; // walk exhausted: the displaced entry is dropped
            k = evicted;
            kgen = vgen;
            slots(k, idx);
            for (int w = 0; w < WAYS; ++w) // don't bounce straight back
                if (idx[w] == vi) idx[w] = idx[(w + 1) % WAYS];
        }
    }

    // Entries that are present and not collectable.
    size_t count_live() const {
        size_t c = 0;
        for (size_t i = 0; i < size; ++i) c += (state[i].load(std::memory_order_relaxed) & (OCC | COLLECT)) == OCC;
        return c;
    }

private:
    void slots(const uint256& k, uint32_t* idx) const {
        const unsigned char* p = k.begin();
        for (int w = 0; w < WAYS; ++w) {
            uint32_t h;
            memcpy(&h, p + 4 * w, 4);
            idx[w] = (uint32_t)(((uint64_t)h * (uint64_t)size) >> 32);
        }
    }
    void place(uint32_t i, const uint256& k, uint8_t gen) {
        keys[i] = k;
        state[i].store((uint8_t)(OCC | gen), std::memory_order_relaxed);
        if (gen) tick();
    }
    // Every so often count the current generation's un-erased entries; once they reach
    // 45% of the table the previous generation becomes collectable and the current
    // one becomes the previous.
    void tick() {
        if (--untilCheck > 0) return;
        size_t live = 0;
        for (size_t i = 0; i < size; ++i)
            live += (state[i].load(std::memory_order_relaxed) & (OCC | COLLECT | GEN)) == (OCC | GEN);
        if (live < genLimit) {
            untilCheck = std::max<size_t>(genLimit - live, genLimit / 16 + 1);
            return;
        }
        for (size_t i = 0; i < size; ++i) {
            const uint8_t st = state[i].load(std::memory_order_relaxed);
            if (!(st & OCC)) continue;
            state[i].store((st & GEN) ? (uint8_t)(st & ~GEN) : (uint8_t)(st | COLLECT), std::memory_order_relaxed);
        }
        untilCheck = genLimit;
    }

    std::vector<uint256> keys;
    std::unique_ptr<std::atomic<uint8_t>[]> state;
    size_t size = 0;
    unsigned depth = 1;
    size_t genLimit = 1;
    ptrdiff_t untilCheck = 1;
    uint32_t rot = 0;
};

// Reader/writer wrapper: contains() under a shared lock, insert/setup exclusive.
class SharedCuckooSet {
public:
    size_t setup_bytes(size_t bytes) {
        std::unique_lock<std::shared_mutex> l(m);
        return set.setup_bytes(bytes);
    }
    bool contains(const uint256& k, bool erase) const {
        std::shared_lock<std::shared_mutex> l(m);
        return set.contains(k, erase);
    }
    void insert(const uint256& k) {
        std::unique_lock<std::shared_mutex> l(m);
        set.insert(k);
    }
    // contains() of n keys under one shared acquisition: many threads probing a block's worth
    // of entries one lock round trip each would serialise on the lock's cache line.
    void contains_many(const uint256* k, size_t n, bool erase, uint8_t* out) const {
        std::shared_lock<std::shared_mutex> l(m);
        for (size_t i = 0; i < n; i++) out[i] = set.contains(k[i], erase);
    }
    size_t capacity() const {
        std::shared_lock<std::shared_mutex> l(m);
        return set.capacity();
    }
    size_t count_live() const {
        std::shared_lock<std::shared_mutex> l(m);
        return set.count_live();
    }

private:
    mutable std::shared_mutex m;
    CuckooHashSet set;
};

} // namespace bcp
