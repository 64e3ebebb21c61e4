// Map keyed by POINTERS, ordered and looked up by the pointed-to values (reference
// src/indirectmap.h:24). The mempool's mapNextTx uses it so each spent outpoint is stored once,
// inside the spending transaction, instead of being copied into the index.
#pragma once
#include <map>

namespace bcp {

template <class K, class T> class indirectmap {
private:
    struct DereferencingComparator {
        bool operator()(const K* a, const K* b) const { return *a < *b; }
    };
    typedef std::map<const K*, T, DereferencingComparator> base;
    base m;

public:
    typedef typename base::iterator iterator;
    typedef typename base::const_iterator const_iterator;
    typedef typename base::size_type size_type;
    typedef typename base::value_type value_type;

    std::pair<iterator, bool> insert(const value_type& value) { return m.insert(value); }
    iterator find(const K& key) { return m.find(&key); }
    const_iterator find(const K& key) const { return m.find(&key); }
    iterator lower_bound(const K& key) { return m.lower_bound(&key); }
    const_iterator lower_bound(const K& key) const { return m.lower_bound(&key); }
    size_type erase(const K& key) { return m.erase(&key); }
    iterator erase(iterator it) { return m.erase(it); }
    size_type count(const K& key) const { return m.count(&key); }

    bool empty() const { return m.empty(); }
    size_type size() const { return m.size(); }
    void clear() { m.clear(); }
    iterator begin() { return m.begin(); }
    iterator end() { return m.end(); }
    const_iterator begin() const { return m.begin(); }
    const_iterator end() const { return m.end(); }
};

} // namespace bcp
