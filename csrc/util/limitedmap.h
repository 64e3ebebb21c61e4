// Size-bounded map that evicts its smallest VALUES when full (reference src/limitedmap.h:14).
// Used for mapAlreadyAskedFor: txid -> earliest request time; once nMaxSize entries exist, a new
// insertion first drops the entry with the lowest (oldest) request time.
#pragma once
#include <cassert>
#include <map>

namespace bcp {

template <typename K, typename V> class limitedmap {
public:
    typedef std::map<K, V> Map;
    typedef typename Map::const_iterator const_iterator;
    typedef typename Map::size_type size_type;

    explicit limitedmap(size_type nMaxSizeIn) : nMaxSize(nMaxSizeIn) { assert(nMaxSizeIn > 0); }

    const_iterator begin() const { return map.begin(); }
    const_iterator end() const { return map.end(); }
    size_type size() const { return map.size(); }
    bool empty() const { return map.empty(); }
    const_iterator find(const K& k) const { return map.find(k); }
    size_type count(const K& k) const { return map.count(k); }

    void insert(const std::pair<K, V>& kv) {
        auto ret = map.insert(kv);
        if (!ret.second) return;
        if (map.size() > nMaxSize) evict_one(ret.first);
        byValue.insert({kv.second, ret.first});
    }
    void erase(const K& k) {
        auto it = map.find(k);
        if (it == map.end()) return;
        unindex(it);
        map.erase(it);
    }
    // change the value of an existing entry
    void update(const_iterator itIn, const V& v) {
        auto it = map.find(itIn->first); // mutable iterator to the same node
        unindex(it);
        it->second = v;
        byValue.insert({v, it});
    }
    size_type max_size() const { return nMaxSize; }
    size_type max_size(size_type s) {
        assert(s > 0);
        nMaxSize = s;
        while (map.size() > nMaxSize) {
            auto victim = byValue.begin();
            map.erase(victim->second);
            byValue.erase(victim);
        }
        return nMaxSize;
    }
    void clear() {
        map.clear();
        byValue.clear();
    }

private:
    typedef typename Map::iterator iterator;
    void unindex(iterator it) {
        auto range = byValue.equal_range(it->second);
        for (auto j = range.first; j != range.second; ++j)
            if (j->second == it) {
                byValue.erase(j);
                return;
            }
        assert(false && "limitedmap: value index out of sync");
    }
    // drop the smallest-valued entry other than the one just inserted
    void evict_one(iterator keep) {
        for (auto j = byValue.begin(); j != byValue.end(); ++j)
            if (j->second != keep) {
                map.erase(j->second);
                byValue.erase(j);
                return;
            }
    }
    Map map;
    std::multimap<V, iterator> byValue;
    size_type nMaxSize;
};

} // namespace bcp
