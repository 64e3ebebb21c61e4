// allocator_tests: the secure-memory Arena (16-byte rounding, coalescing back to one free
// chunk, double-free detection, exhaustion, interleaved pseudo-random alloc/free) over a
// synthetic address range; LockedPool over a mock page allocator (arena growth, the locked
// byte count when only one of three arenas locks, refusal of 0-byte and over-arena requests);
// and the live LockedPoolManager.
// Parity: reference src/test/allocator_tests.cpp (arena_tests, lockedpool_tests_mock,
// lockedpool_tests_live).
#include "test/unittest.h"

#include "util/lockedpool.h"

#include <limits>
#include <stdexcept>

using namespace bcp;

TEST_CASE(allocator_tests, arena_tests) {
    // a fake base address: the arena only does bookkeeping, it never touches the memory
    void* synth_base = reinterpret_cast<void*>(0x08000000);
    const size_t synth_size = 1024 * 1024;
    Arena b(synth_base, synth_size, 16);
    void* chunk = b.alloc(1000);
    CHECK(chunk != nullptr);
    CHECK_EQ(b.stats().used, (size_t)1008); // rounded to 16
    CHECK_EQ(b.stats().total, synth_size);
    b.free(chunk);
    CHECK_EQ(b.stats().used, (size_t)0);
    CHECK_EQ(b.stats().free, synth_size);
    CHECK_THROWS(b.free(chunk)); // double free

    void* a0 = b.alloc(128);
    void* a1 = b.alloc(256);
    void* a2 = b.alloc(512);
    CHECK_EQ(b.stats().used, (size_t)896);
    CHECK_EQ(b.stats().total, synth_size);
    b.free(a0);
    CHECK_EQ(b.stats().used, (size_t)768);
    b.free(a1);
    CHECK_EQ(b.stats().used, (size_t)512);
    void* a3 = b.alloc(128);
    CHECK_EQ(b.stats().used, (size_t)640);
    b.free(a2);
    CHECK_EQ(b.stats().used, (size_t)128);
    b.free(a3);
    CHECK_EQ(b.stats().used, (size_t)0);
    CHECK_EQ(b.stats().chunks_used, (size_t)0);
    CHECK_EQ(b.stats().total, synth_size);
    CHECK_EQ(b.stats().free, synth_size);
    CHECK_EQ(b.stats().chunks_free, (size_t)1);

    std::vector<void*> addr;
    CHECK(b.alloc(0) == nullptr);
    for (int x = 0; x < 1024; ++x) addr.push_back(b.alloc(1024)); // fill it
    CHECK_EQ(b.stats().free, (size_t)0);
    CHECK(b.alloc(1024) == nullptr);
    CHECK(b.alloc(0) == nullptr);
    for (int x = 0; x < 1024; ++x) b.free(addr[x]);
    addr.clear();
    CHECK_EQ(b.stats().total, synth_size);
    CHECK_EQ(b.stats().free, synth_size);
    for (int x = 0; x < 1024; ++x) addr.push_back(b.alloc(1024)); // and freed in reverse
    for (int x = 0; x < 1024; ++x) b.free(addr[1023 - x]);
    addr.clear();
    // unequal sizes, freed out of order (some allocations fail: freeing nullptr is allowed)
    for (int x = 0; x < 2048; ++x) addr.push_back(b.alloc(x + 1));
    for (int x = 0; x < 2048; ++x) b.free(addr[((x * 23) % 2048) ^ 242]);
    addr.clear();
    // interleaved alloc/free driven by an LFSR
    addr.assign(2048, nullptr);
    uint32_t s = 0x12345678;
    for (int x = 0; x < 5000; ++x) {
        const int idx = s & (addr.size() - 1);
        if (s & 0x80000000) {
            b.free(addr[idx]);
            addr[idx] = nullptr;
        } else if (!addr[idx]) {
            addr[idx] = b.alloc((s >> 16) & 2047);
        }
        const bool lsb = s & 1;
        s >>= 1;
        if (lsb) s ^= 0xf00f00f0; // period 0xf7ffffe0
    }
    for (void* p : addr) b.free(p);
    CHECK_EQ(b.stats().total, synth_size);
    CHECK_EQ(b.stats().free, synth_size);
}

namespace {

// hands out `count` fake arenas, the first `lockedcount` of them "locked"
class TestLockedPageAllocator : public LockedPageAllocator {
public:
    TestLockedPageAllocator(int count_in, int lockedcount_in) : count(count_in), lockedcount(lockedcount_in) {}
    void* AllocateLocked(size_t, bool* lockingSuccess) override {
        *lockingSuccess = false;
        if (count > 0) {
            --count;
            if (lockedcount > 0) {
                --lockedcount;
                *lockingSuccess = true;
            }
            return reinterpret_cast<void*>(0x08000000 + ((uintptr_t)count << 24)); // never dereferenced
        }
        return nullptr;
    }
    void FreeLocked(void*, size_t) override {}
    size_t GetLimit() override { return std::numeric_limits<size_t>::max(); }

private:
    int count, lockedcount;
};

} // namespace

TEST_CASE(allocator_tests, lockedpool_tests_mock) {
    LockedPool pool(std::unique_ptr<LockedPageAllocator>(new TestLockedPageAllocator(3, 1)));
    CHECK_EQ(pool.stats().total, (size_t)0);
    CHECK_EQ(pool.stats().locked, (size_t)0);
    CHECK(pool.alloc(0) == nullptr); // refused without creating an arena
    CHECK_EQ(pool.stats().used, (size_t)0);
    CHECK_EQ(pool.stats().free, (size_t)0);
    CHECK(pool.alloc(LockedPool::ARENA_SIZE + 1) == nullptr);
    CHECK_EQ(pool.stats().used, (size_t)0);
    CHECK_EQ(pool.stats().free, (size_t)0);

    void* a0 = pool.alloc(LockedPool::ARENA_SIZE / 2);
    CHECK(a0);
    CHECK_EQ(pool.stats().locked, LockedPool::ARENA_SIZE);
    void* a[5];
    for (void*& p : a) {
        p = pool.alloc(LockedPool::ARENA_SIZE / 2);
        CHECK(p);
    }
    CHECK(!pool.alloc(16)); // three arenas, all full
    pool.free(a0);
    pool.free(a[1]);
    pool.free(a[3]);
    pool.free(a[0]);
    pool.free(a[2]);
    pool.free(a[4]);
    CHECK_EQ(pool.stats().total, 3 * LockedPool::ARENA_SIZE);
    CHECK_EQ(pool.stats().locked, LockedPool::ARENA_SIZE);
    CHECK_EQ(pool.stats().used, (size_t)0);
}

TEST_CASE(allocator_tests, lockedpool_tests_live) {
    LockedPoolManager& pool = LockedPoolManager::Instance();
    const LockedPool::Stats initial = pool.stats();
    void* a0 = pool.alloc(16);
    REQUIRE(a0);
    *static_cast<uint32_t*>(a0) = 0x1234;
    CHECK_EQ(*static_cast<uint32_t*>(a0), (uint32_t)0x1234);
    pool.free(a0);
    CHECK_THROWS(pool.free(a0));
    CHECK(pool.stats().total <= initial.total + LockedPool::ARENA_SIZE);
    CHECK_EQ(pool.stats().used, initial.used);
}
