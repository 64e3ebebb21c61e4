// Node arena for the UTXO cache's hash map (the role of reference src/support/allocators/
// pool.h in later releases; the reference at this version uses plain std::allocator).
// Every entry of a CCoinsViewCache is one hash-map node; a block's connect adds and removes
// about one node per input and output (84k for an 8 MB block), and the per-block view is freed
// node by node afterwards. Carving the nodes out of 256 KiB chunks and recycling them through a
// free list per size class takes malloc/free off that path and keeps a block's nodes adjacent.
//
// One arena per container: it is not thread-safe, exactly like the container it serves. Copies
// of an allocator (the container's rebinds) share the arena; a copied container gets a fresh one.
#pragma once
#include <cstddef>
#include <memory>
#include <new>
#include <type_traits>
#include <vector>

namespace bcp {

class NodeArena {
public:
    static constexpr size_t MAX_NODE = 256; // larger requests go to operator new
    static constexpr size_t ALIGN = 16;
    static constexpr size_t CHUNK = 256 << 10;

    NodeArena() = default;
    NodeArena(const NodeArena&) = delete;
    NodeArena& operator=(const NodeArena&) = delete;
    ~NodeArena() {
        for (void* c : chunks) ::operator delete(c);
    }

    static bool Serves(size_t bytes, size_t align) { return bytes <= MAX_NODE && align <= ALIGN; }

    void* Allocate(size_t bytes) {
        const size_t cls = (bytes + ALIGN - 1) / ALIGN; // 1..16
        if (FreeNode* f = freeList[cls]) {
            freeList[cls] = f->next;
            return f;
        }
        const size_t sz = cls * ALIGN;
        if (left < sz) {
            cur = static_cast<char*>(::operator new(CHUNK));
            chunks.push_back(cur);
            left = CHUNK;
        }
        void* p = cur;
        cur += sz;
        left -= sz;
        return p;
    }
    void Free(void* p, size_t bytes) {
        const size_t cls = (bytes + ALIGN - 1) / ALIGN;
        FreeNode* f = static_cast<FreeNode*>(p);
        f->next = freeList[cls];
        freeList[cls] = f;
    }
    // bytes held from the system (whole chunks, used or not)
    size_t ChunkBytes() const { return chunks.size() * CHUNK; }

private:
    struct FreeNode {
        FreeNode* next;
    };
    FreeNode* freeList[MAX_NODE / ALIGN + 1] = {};
    std::vector<void*> chunks;
    char* cur = nullptr;
    size_t left = 0;
};

template <typename T> class NodePoolAllocator {
public:
    using value_type = T;
    using propagate_on_container_copy_assignment = std::true_type;
    using propagate_on_container_move_assignment = std::true_type;
    using propagate_on_container_swap = std::true_type;
    using is_always_equal = std::false_type;

    NodePoolAllocator() : arena(std::make_shared<NodeArena>()) {}
    template <typename U> NodePoolAllocator(const NodePoolAllocator<U>& o) noexcept : arena(o.arena) {}

    T* allocate(size_t n) {
        if (n == 1 && NodeArena::Serves(sizeof(T), alignof(T))) return static_cast<T*>(arena->Allocate(sizeof(T)));
        return static_cast<T*>(::operator new(n * sizeof(T)));
    }
    void deallocate(T* p, size_t n) noexcept {
        if (n == 1 && NodeArena::Serves(sizeof(T), alignof(T))) arena->Free(p, sizeof(T));
        else ::operator delete(p);
    }
    // a copied container gets an arena of its own (the copy may outlive or be used apart from
    // the original)
    NodePoolAllocator select_on_container_copy_construction() const { return NodePoolAllocator(); }

    // bytes the arena holds from the system (chunks, live nodes and free-list slack alike)
    size_t ArenaBytes() const { return arena->ChunkBytes(); }

    template <typename U> bool operator==(const NodePoolAllocator<U>& o) const noexcept { return arena == o.arena; }
    template <typename U> bool operator!=(const NodePoolAllocator<U>& o) const noexcept { return arena != o.arena; }

private:
    template <typename U> friend class NodePoolAllocator;
    std::shared_ptr<NodeArena> arena;
};

} // namespace bcp
