// Heap-usage model for in-memory containers (reference src/memusage.h, src/core_memusage.h).
// Sizes the mempool (-maxmempool) and the UTXO cache (-dbcache) by what the allocator really
// hands out, not by element counts: glibc malloc on 64-bit rounds every request plus its
// 8-byte chunk header up to a 16-byte multiple, with a 32-byte minimum chunk.
#pragma once
#include "util/prevector.h"
#include <cstddef>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace bcp {
namespace memusage {

inline size_t MallocUsage(size_t alloc) {
    if (alloc == 0) return 0;
    const size_t chunk = (alloc + 8 + 15) & ~(size_t)15;
    return chunk < 32 ? 32 : chunk;
}

// Node layouts of the libstdc++ containers: red-black tree nodes carry a color word and three
// pointers; hash-table nodes a next pointer and the cached hash.
struct stl_tree_node {
    int color;
    void *parent, *left, *right;
};
struct stl_hash_node {
    void* next;
    size_t hash;
};

template <unsigned N, typename X> inline size_t DynamicUsage(const prevector<N, X>& v) {
    return MallocUsage(v.allocated_memory());
}
template <typename X> inline size_t DynamicUsage(const std::vector<X>& v) {
    return MallocUsage(v.capacity() * sizeof(X));
}
inline size_t DynamicUsage(const std::string& s) {
    return s.capacity() > 15 ? MallocUsage(s.capacity() + 1) : 0; // small-string buffer inline
}
template <typename X, typename Y> inline size_t DynamicUsage(const std::set<X, Y>& s) {
    return MallocUsage(sizeof(stl_tree_node) + sizeof(X)) * s.size();
}
template <typename X, typename Y> inline size_t IncrementalDynamicUsage(const std::set<X, Y>&) {
    return MallocUsage(sizeof(stl_tree_node) + sizeof(X));
}
template <typename X, typename Y, typename Z> inline size_t DynamicUsage(const std::map<X, Y, Z>& m) {
    return MallocUsage(sizeof(stl_tree_node) + sizeof(std::pair<const X, Y>)) * m.size();
}
template <typename X, typename Y, typename Z> inline size_t IncrementalDynamicUsage(const std::map<X, Y, Z>&) {
    return MallocUsage(sizeof(stl_tree_node) + sizeof(std::pair<const X, Y>));
}
template <typename X, typename Y, typename Z> inline size_t DynamicUsage(const std::multimap<X, Y, Z>& m) {
    return MallocUsage(sizeof(stl_tree_node) + sizeof(std::pair<const X, Y>)) * m.size();
}
template <typename X, typename Y, typename Z> inline size_t DynamicUsage(const std::unordered_set<X, Y, Z>& s) {
    return MallocUsage(sizeof(stl_hash_node) + sizeof(X)) * s.size() + MallocUsage(sizeof(void*) * s.bucket_count());
}
template <typename X, typename Y, typename Z, typename W, typename A>
inline size_t DynamicUsage(const std::unordered_map<X, Y, Z, W, A>& m) {
    return MallocUsage(sizeof(stl_hash_node) + sizeof(std::pair<const X, Y>)) * m.size() +
           MallocUsage(sizeof(void*) * m.bucket_count());
}
// an object made with make_shared: one block holding the control block and the object
template <typename X> inline size_t DynamicUsage(const std::shared_ptr<X>& p) {
    return p ? MallocUsage(sizeof(X) + 2 * sizeof(long) + sizeof(void*)) : 0;
}
template <typename X> inline size_t DynamicUsage(const std::unique_ptr<X>& p) {
    return p ? MallocUsage(sizeof(X)) : 0;
}

} // namespace memusage
} // namespace bcp
