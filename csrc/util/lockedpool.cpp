#include "util/lockedpool.h"

#include <sys/mman.h>
#include <sys/resource.h>
#include <unistd.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <stdexcept>

namespace bcp {

void memory_cleanse(void* ptr, size_t len) {
    std::memset(ptr, 0, len);
    // compiler barrier: the memset above must not be removed as a dead store
    __asm__ __volatile__("" : : "r"(ptr) : "memory");
}

static inline size_t align_up(size_t x, size_t align) { return (x + align - 1) & ~(align - 1); }

// ------------------------------------------------------------------ Arena
Arena::Arena(void* base_in, size_t size_in, size_t alignment_in)
    : base(static_cast<char*>(base_in)), end(static_cast<char*>(base_in) + size_in), alignment(alignment_in) {
    auto it = size_to_free_chunk.emplace(size_in, base);
    chunks_free.emplace(base, it);
    chunks_free_end.emplace(base + size_in, it);
}

Arena::~Arena() {}

void* Arena::alloc(size_t size) {
    size = align_up(size, alignment);
    if (size == 0) return nullptr;
    // best fit: smallest free chunk that is large enough
    auto sit = size_to_free_chunk.lower_bound(size);
    if (sit == size_to_free_chunk.end()) return nullptr;
    const size_t chunkSize = sit->first;
    char* const chunk = sit->second;
    // carve from the end of the free chunk so the free entry keeps its start
    char* const alloced = chunk + chunkSize - size;
    chunks_free_end.erase(chunk + chunkSize);
    size_to_free_chunk.erase(sit);
    if (chunkSize > size) {
        auto it = size_to_free_chunk.emplace(chunkSize - size, chunk);
        chunks_free[chunk] = it;
        chunks_free_end.emplace(chunk + chunkSize - size, it);
    } else {
        chunks_free.erase(chunk);
    }
    chunks_used.emplace(alloced, size);
    return alloced;
}

void Arena::free(void* ptr) {
    if (ptr == nullptr) return;
    auto i = chunks_used.find(static_cast<char*>(ptr));
    if (i == chunks_used.end()) throw std::runtime_error("Arena: invalid or double free");
    std::pair<char*, size_t> freed = *i;
    chunks_used.erase(i);
    // coalesce with the preceding free chunk
    auto prev = chunks_free_end.find(freed.first);
    if (prev != chunks_free_end.end()) {
        freed.first -= prev->second->first;
        freed.second += prev->second->first;
        size_to_free_chunk.erase(prev->second);
        chunks_free_end.erase(prev);
    }
    // and the following one
    auto next = chunks_free.find(freed.first + freed.second);
    if (next != chunks_free.end()) {
        freed.second += next->second->first;
        chunks_free_end.erase(freed.first + freed.second);
        size_to_free_chunk.erase(next->second);
        chunks_free.erase(next);
    }
    auto it = size_to_free_chunk.emplace(freed.second, freed.first);
    chunks_free[freed.first] = it;
    chunks_free_end[freed.first + freed.second] = it;
}

Arena::Stats Arena::stats() const {
    Stats r{0, 0, 0, chunks_used.size(), chunks_free.size()};
    for (const auto& kv : chunks_used) r.used += kv.second;
    for (const auto& kv : chunks_free) r.free += kv.second->first;
    r.total = r.used + r.free;
    return r;
}

// ------------------------------------------------------------------ page allocator
PosixLockedPageAllocator::PosixLockedPageAllocator() {
    const long ps = sysconf(_SC_PAGESIZE);
    page_size = ps > 0 ? (size_t)ps : 4096;
}

void* PosixLockedPageAllocator::AllocateLocked(size_t len, bool* lockingSuccess) {
    len = align_up(len, page_size);
    void* addr = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (addr == MAP_FAILED) return nullptr;
    *lockingSuccess = mlock(addr, len) == 0;
#ifdef MADV_DONTDUMP
    madvise(addr, len, MADV_DONTDUMP); // keep secrets out of core dumps
#endif
    return addr;
}

void PosixLockedPageAllocator::FreeLocked(void* addr, size_t len) {
    len = align_up(len, page_size);
    memory_cleanse(addr, len);
    munlock(addr, len);
    munmap(addr, len);
}

size_t PosixLockedPageAllocator::GetLimit() {
    struct rlimit rlim;
    if (getrlimit(RLIMIT_MEMLOCK, &rlim) == 0 && rlim.rlim_cur != RLIM_INFINITY) return rlim.rlim_cur;
    return SIZE_MAX;
}

// ------------------------------------------------------------------ LockedPool
LockedPool::LockedPool(std::unique_ptr<LockedPageAllocator> allocator_in, LockingFailed_Callback cb)
    : allocator(std::move(allocator_in)), lf_cb(cb) {}

LockedPool::~LockedPool() {}

void* LockedPool::alloc(size_t size) {
    std::lock_guard<std::mutex> l(mutex);
    if (size == 0 || size > ARENA_SIZE) return nullptr;
    for (auto& arena : arenas)
        if (void* p = arena.alloc(size)) return p;
    if (new_arena(ARENA_SIZE, ARENA_ALIGN)) return arenas.back().alloc(size);
    return nullptr;
}

void LockedPool::free(void* ptr) {
    std::lock_guard<std::mutex> l(mutex);
    for (auto& arena : arenas)
        if (arena.addressInArena(ptr)) {
            arena.free(ptr);
            return;
        }
    throw std::runtime_error("LockedPool: invalid address not pointing to any arena");
}

LockedPool::Stats LockedPool::stats() const {
    std::lock_guard<std::mutex> l(mutex);
    Stats r{0, 0, 0, cumulative_bytes_locked, 0, 0};
    for (const auto& arena : arenas) {
        const Arena::Stats s = arena.stats();
        r.used += s.used;
        r.free += s.free;
        r.total += s.total;
        r.chunks_used += s.chunks_used;
        r.chunks_free += s.chunks_free;
    }
    return r;
}

bool LockedPool::new_arena(size_t size, size_t align) {
    bool locked = false;
    // the first arena is clipped to the process lock limit so it at least gets locked
    if (arenas.empty()) {
        const size_t limit = allocator->GetLimit();
        if (limit > 0) size = std::min(size, limit);
    }
    void* addr = allocator->AllocateLocked(size, &locked);
    if (!addr) return false;
    if (locked) {
        cumulative_bytes_locked += size;
    } else if (lf_cb && !lf_cb()) {
        allocator->FreeLocked(addr, size);
        return false;
    }
    arenas.emplace_back(allocator.get(), addr, size, align);
    return true;
}

LockedPool::LockedPageArena::LockedPageArena(LockedPageAllocator* alloc, void* base_in, size_t size_in, size_t align)
    : Arena(base_in, size_in, align), base(base_in), size(size_in), allocator(alloc) {}

LockedPool::LockedPageArena::~LockedPageArena() { allocator->FreeLocked(base, size); }

// ------------------------------------------------------------------ manager
LockedPoolManager::LockedPoolManager(std::unique_ptr<LockedPageAllocator> a) : LockedPool(std::move(a), &LockingFailed) {}

bool LockedPoolManager::LockingFailed() {
    // mlock may be unavailable (containers, RLIMIT_MEMLOCK): keep working with unlocked pages
    return true;
}

LockedPoolManager& LockedPoolManager::Instance() {
    // intentionally leaked: secure allocations may outlive static destructors
    static LockedPoolManager* inst = new LockedPoolManager(std::unique_ptr<LockedPageAllocator>(new PosixLockedPageAllocator()));
    return *inst;
}

} // namespace bcp
