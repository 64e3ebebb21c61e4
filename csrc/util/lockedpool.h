// Secure memory for key material.
// Parity: reference src/support/lockedpool.{h,cpp} (Arena: best-fit allocation inside a
// fixed region with chunk coalescing; LockedPool: grows by 256 KiB arenas obtained from
// a LockedPageAllocator that mlock()s pages and tolerates lock failure; stats
// used/free/total/locked/chunks_used/chunks_free; LockedPoolManager singleton),
// src/support/allocators/secure.h (secure_allocator: cleanse on free) and
// src/support/cleanse.cpp (memory_cleanse that the optimiser cannot elide).
#pragma once
#include <cstddef>
#include <cstdint>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace bcp {

void memory_cleanse(void* ptr, size_t len);

class LockedPageAllocator {
public:
    virtual ~LockedPageAllocator() {}
    // Allocate len bytes of page-aligned memory and try to lock it; lockingSuccess reports mlock.
    virtual void* AllocateLocked(size_t len, bool* lockingSuccess) = 0;
    virtual void FreeLocked(void* addr, size_t len) = 0;
    virtual size_t GetLimit() = 0; // RLIMIT_MEMLOCK (or SIZE_MAX)
};

class PosixLockedPageAllocator : public LockedPageAllocator {
public:
    PosixLockedPageAllocator();
    void* AllocateLocked(size_t len, bool* lockingSuccess) override;
    void FreeLocked(void* addr, size_t len) override;
    size_t GetLimit() override;

private:
    size_t page_size;
};

class Arena {
public:
    Arena(void* base, size_t size, size_t alignment);
    virtual ~Arena();
    Arena(const Arena&) = delete;
    struct Stats {
        size_t used, free, total, chunks_used, chunks_free;
    };
    void* alloc(size_t size);
    void free(void* ptr);
    Stats stats() const;
    bool addressInArena(void* ptr) const { return ptr >= base && ptr < end; }

private:
    typedef std::multimap<size_t, char*> SizeToChunkSortedMap;
    SizeToChunkSortedMap size_to_free_chunk;
    typedef std::unordered_map<char*, SizeToChunkSortedMap::const_iterator> ChunkToSizeMap;
    ChunkToSizeMap chunks_free;     // begin -> size map entry
    ChunkToSizeMap chunks_free_end; // end -> size map entry
    std::unordered_map<char*, size_t> chunks_used;
    char* base;
    char* end;
    size_t alignment;
};

class LockedPool {
public:
    static const size_t ARENA_SIZE = 256 * 1024;
    static const size_t ARENA_ALIGN = 16;
    typedef bool (*LockingFailed_Callback)();
    struct Stats {
        size_t used, free, total, locked, chunks_used, chunks_free;
    };
    explicit LockedPool(std::unique_ptr<LockedPageAllocator> allocator, LockingFailed_Callback cb = nullptr);
    ~LockedPool();
    void* alloc(size_t size);
    void free(void* ptr);
    Stats stats() const;

private:
    class LockedPageArena : public Arena {
    public:
        LockedPageArena(LockedPageAllocator* alloc, void* base, size_t size, size_t align);
        ~LockedPageArena();

    private:
        void* base;
        size_t size;
        LockedPageAllocator* allocator;
    };
    bool new_arena(size_t size, size_t align);
    std::unique_ptr<LockedPageAllocator> allocator;
    std::list<LockedPageArena> arenas;
    LockingFailed_Callback lf_cb;
    size_t cumulative_bytes_locked = 0;
    mutable std::mutex mutex;
};

// Process-wide pool for secure allocations.
class LockedPoolManager : public LockedPool {
public:
    static LockedPoolManager& Instance();

private:
    explicit LockedPoolManager(std::unique_ptr<LockedPageAllocator> allocator);
    static bool LockingFailed();
};

template <typename T> struct secure_allocator {
    typedef T value_type;
    secure_allocator() noexcept {}
    template <typename U> secure_allocator(const secure_allocator<U>&) noexcept {}
    T* allocate(std::size_t n) {
        T* p = static_cast<T*>(LockedPoolManager::Instance().alloc(sizeof(T) * n));
        if (!p) throw std::bad_alloc();
        return p;
    }
    void deallocate(T* p, std::size_t n) {
        if (p) {
            memory_cleanse(p, sizeof(T) * n);
            LockedPoolManager::Instance().free(p);
        }
    }
    template <typename U> struct rebind { typedef secure_allocator<U> other; };
    template <typename U> bool operator==(const secure_allocator<U>&) const noexcept { return true; }
    template <typename U> bool operator!=(const secure_allocator<U>&) const noexcept { return false; }
};

typedef std::basic_string<char, std::char_traits<char>, secure_allocator<char>> SecureString;

} // namespace bcp
