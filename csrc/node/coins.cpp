#include "node/coins.h"

#include <algorithm>
#include "util/memusage.h"
#include "util/reaper.h"
#include "keys/key.h"
#include "secp256k1/secp256k1.h"

#include <cassert>
#include <cstring>
#include <mutex>

namespace bcp {

// ------------------------------------------------------------------ amount compression
uint64_t CompressAmount(uint64_t n) {
    if (n == 0) return 0;
    int e = 0;
    while ((n % 10) == 0 && e < 9) {
        n /= 10;
        e++;
    }
    if (e < 9) {
        const int d = (int)(n % 10);
        n /= 10;
        return 1 + (n * 9 + d - 1) * 10 + e;
    }
    return 1 + (n - 1) * 10 + 9;
}

uint64_t DecompressAmount(uint64_t x) {
    if (x == 0) return 0;
    x--;
    int e = (int)(x % 10);
    x /= 10;
    uint64_t n = 0;
    if (e < 9) {
        const int d = (int)(x % 9) + 1;
        x /= 9;
        n = x * 10 + d;
    } else {
        n = x + 1;
    }
    while (e) {
        n *= 10;
        e--;
    }
    return n;
}

// ------------------------------------------------------------------ script compression
bool CompressScript(const CScript& s, std::vector<unsigned char>& out) {
    if (s.size() == 25 && s[0] == OP_DUP && s[1] == OP_HASH160 && s[2] == 20 && s[23] == OP_EQUALVERIFY &&
        s[24] == OP_CHECKSIG) {
        out.assign(21, 0);
        memcpy(&out[1], &s[3], 20);
        return true;
    }
    if (s.size() == 23 && s[0] == OP_HASH160 && s[1] == 20 && s[22] == OP_EQUAL) {
        out.assign(21, 1);
        memcpy(&out[1], &s[2], 20);
        return true;
    }
    if (s.size() == 35 && s[0] == 33 && s[34] == OP_CHECKSIG && (s[1] == 0x02 || s[1] == 0x03)) {
        out.assign(33, s[1]);
        memcpy(&out[1], &s[2], 32);
        return true;
    }
    if (s.size() == 67 && s[0] == 65 && s[66] == OP_CHECKSIG && s[1] == 0x04) {
        CPubKey pk(s.begin() + 1, s.begin() + 66);
        if (!pk.IsFullyValid()) return false; // only valid keys can be re-derived from x
        out.assign(33, 0x04 | (s[65] & 0x01));
        memcpy(&out[1], &s[2], 32);
        return true;
    }
    return false;
}

unsigned GetSpecialScriptSize(unsigned nSize) {
    if (nSize == 0 || nSize == 1) return 20;
    if (nSize >= 2 && nSize <= 5) return 32;
    return 0;
}

bool DecompressScript(CScript& s, unsigned nSize, const std::vector<unsigned char>& in) {
    switch (nSize) {
    case 0:
        s.resize(25);
        s[0] = OP_DUP;
        s[1] = OP_HASH160;
        s[2] = 20;
        memcpy(&s[3], in.data(), 20);
        s[23] = OP_EQUALVERIFY;
        s[24] = OP_CHECKSIG;
        return true;
    case 1:
        s.resize(23);
        s[0] = OP_HASH160;
        s[1] = 20;
        memcpy(&s[2], in.data(), 20);
        s[22] = OP_EQUAL;
        return true;
    case 2:
    case 3:
        s.resize(35);
        s[0] = 33;
        s[1] = (unsigned char)nSize;
        memcpy(&s[2], in.data(), 32);
        s[34] = OP_CHECKSIG;
        return true;
    case 4:
    case 5: {
        unsigned char vch[33];
        vch[0] = (unsigned char)(nSize - 2);
        memcpy(&vch[1], in.data(), 32);
        CPubKey pk(vch, vch + 33);
        if (!pk.Decompress()) return false;
        s.resize(67);
        s[0] = 65;
        memcpy(&s[1], pk.begin(), 65);
        s[66] = OP_CHECKSIG;
        return true;
    }
    }
    return false;
}

// ------------------------------------------------------------------ cache
SaltedOutpointHasher::SaltedOutpointHasher() {
    static const std::pair<uint64_t, uint64_t> salt = [] {
        uint64_t a, b;
        GetRandBytes((unsigned char*)&a, 8);
        GetRandBytes((unsigned char*)&b, 8);
        return std::make_pair(a, b);
    }();
    k0 = salt.first;
    k1 = salt.second;
}

CCoinsViewCache::CCoinsViewCache(CCoinsView* b) : CCoinsViewBacked(b) {}

size_t CCoinsViewCache::DynamicMemoryUsage() const {
    // hash-table nodes and buckets plus the scripts' heap buffers (reference coins.cpp). The
    // nodes live in each shard's NodeArena, which keeps its chunks (and the free-list slack in
    // them) after entries are erased or the cache is flushed: the node share is whichever is
    // larger, the live nodes' estimate or the chunk bytes the arena holds, so -dbcache sees
    // the memory the process really keeps.
    size_t n = CachedCoinsUsage();
    for (unsigned s = 0; s < CCoinsMap::SHARDS; s++) {
        const auto& sh = cacheCoins.shard(s);
        const size_t buckets = memusage::MallocUsage(sizeof(void*) * sh.bucket_count());
        const size_t nodes = memusage::DynamicUsage(sh) - buckets;
        n += buckets + std::max(nodes, sh.get_allocator().ArenaBytes());
    }
    return n;
}

CCoinsMap::iterator CCoinsViewCache::FetchCoin(const COutPoint& outpoint) const {
    auto it = cacheCoins.find(outpoint);
    if (it != cacheCoins.end()) return it;
    Coin tmp;
    if (!base->GetCoin(outpoint, tmp)) return cacheCoins.end();
    const unsigned s = CCoinsMap::ShardOf(outpoint);
    auto ret = cacheCoins.shard(s)
                   .emplace(std::piecewise_construct, std::forward_as_tuple(outpoint), std::forward_as_tuple(std::move(tmp)))
                   .first;
    if (ret->second.coin.IsSpent()) {
        // a spent coin in the parent is FRESH from our point of view
        ret->second.flags = CCoinsCacheEntry::FRESH;
    }
    usage[s].bytes += ret->second.coin.DynamicMemoryUsage();
    return CCoinsMap::iterator(&cacheCoins, s, ret);
}

bool CCoinsViewCache::GetCoin(const COutPoint& outpoint, Coin& coin) const {
    auto it = FetchCoin(outpoint);
    if (it == cacheCoins.end()) return false;
    coin = it->second.coin;
    return true; // a spent entry is reported too (callers check IsSpent), so a child cache fetching
                 // it marks its copy FRESH (reference coins.cpp GetCoin/FetchCoin)
}

void CCoinsViewCache::AddCoin(const COutPoint& outpoint, Coin&& coin, bool possible_overwrite) {
    assert(!coin.IsSpent());
    if (coin.out.scriptPubKey.IsUnspendable()) return;
    const unsigned s = CCoinsMap::ShardOf(outpoint);
    auto ins = cacheCoins.shard(s).emplace(std::piecewise_construct, std::forward_as_tuple(outpoint), std::tuple<>());
    auto it = ins.first;
    bool fresh = false;
    if (!ins.second) usage[s].bytes -= it->second.coin.DynamicMemoryUsage();
    if (!possible_overwrite) {
        if (!it->second.coin.IsSpent()) throw std::logic_error("Adding new coin that replaces non-pruned entry");
        fresh = !(it->second.flags & CCoinsCacheEntry::DIRTY);
    }
    it->second.coin = std::move(coin);
    it->second.flags |= CCoinsCacheEntry::DIRTY | (fresh ? CCoinsCacheEntry::FRESH : 0);
    usage[s].bytes += it->second.coin.DynamicMemoryUsage();
}

void AddCoins(CCoinsViewCache& cache, const CTransaction& tx, int nHeight, bool check) {
    const bool fCoinbase = tx.IsCoinBase();
    const uint256& txid = tx.GetHash();
    for (size_t i = 0; i < tx.vout.size(); ++i) {
        const COutPoint op(txid, (uint32_t)i);
        const bool overwrite = check ? cache.HaveCoin(op) : fCoinbase;
        cache.AddCoin(op, Coin(tx.vout[i], nHeight, fCoinbase), overwrite);
    }
}

bool CCoinsViewCache::SpendCoin(const COutPoint& outpoint, Coin* moveout) {
    auto it = FetchCoin(outpoint);
    if (it == cacheCoins.end()) return false;
    const unsigned s = CCoinsMap::ShardOf(outpoint);
    usage[s].bytes -= it->second.coin.DynamicMemoryUsage();
    if (moveout) *moveout = std::move(it->second.coin);
    if (it->second.flags & CCoinsCacheEntry::FRESH) {
        cacheCoins.erase(it);
    } else {
        it->second.flags |= CCoinsCacheEntry::DIRTY;
        it->second.coin.Clear();
    }
    return true;
}

static const Coin coinEmpty;

const Coin& CCoinsViewCache::AccessCoin(const COutPoint& outpoint) const {
    auto it = FetchCoin(outpoint);
    if (it == cacheCoins.end()) return coinEmpty;
    return it->second.coin;
}

void CCoinsViewCache::SpendFetched(const COutPoint& outpoint, Coin&& coin, Coin* moveto) {
    assert(!coin.IsSpent());
    auto ins = cacheCoins.shard(CCoinsMap::ShardOf(outpoint))
                   .emplace(std::piecewise_construct, std::forward_as_tuple(outpoint), std::tuple<>());
    assert(ins.second);
    ins.first->second.flags = CCoinsCacheEntry::DIRTY; // not FRESH: the base holds the coin
    if (moveto) *moveto = std::move(coin);
}

void CCoinsViewCache::SpendFetchedMoved(const COutPoint& outpoint) {
    auto ins = cacheCoins.shard(CCoinsMap::ShardOf(outpoint))
                   .emplace(std::piecewise_construct, std::forward_as_tuple(outpoint), std::tuple<>());
    assert(ins.second);
    ins.first->second.flags = CCoinsCacheEntry::DIRTY; // not FRESH: the base holds the coin
}

void CCoinsViewCache::SpendPeeked(const COutPoint& outpoint) {
    const unsigned s = CCoinsMap::ShardOf(outpoint);
    auto ins = cacheCoins.shard(s).try_emplace(outpoint); // no node is made when the entry exists
    if (ins.second) {
        ins.first->second.flags = CCoinsCacheEntry::DIRTY; // not FRESH: the base holds the coin
        return;
    }
    auto it = ins.first;
    usage[s].bytes -= it->second.coin.DynamicMemoryUsage();
    if (it->second.flags & CCoinsCacheEntry::FRESH) {
        cacheCoins.shard(s).erase(it);
    } else {
        it->second.flags |= CCoinsCacheEntry::DIRTY;
        it->second.coin.Clear();
    }
}

bool CCoinsViewCache::HaveCoin(const COutPoint& outpoint) const {
    auto it = FetchCoin(outpoint);
    return it != cacheCoins.end() && !it->second.coin.IsSpent();
}

bool CCoinsViewCache::PeekCoin(const COutPoint& outpoint, Coin& coin) const {
    auto it = cacheCoins.find(outpoint);
    if (it == cacheCoins.end()) return base->PeekCoin(outpoint, coin);
    coin = it->second.coin; // a spent entry here hides the parent's coin
    return true;
}

void CCoinsViewCache::PeekCoins(const COutPoint* outpoints, size_t n, Coin* coins, uint8_t* found) const {
    std::vector<COutPoint> miss;
    std::vector<size_t> where;
    for (size_t i = 0; i < n; i++) {
        auto it = cacheCoins.find(outpoints[i]);
        if (it != cacheCoins.end()) {
            coins[i] = it->second.coin;
            found[i] = 1;
        } else {
            miss.push_back(outpoints[i]);
            where.push_back(i);
        }
    }
    if (miss.empty()) return;
    std::vector<Coin> got(miss.size());
    std::unique_ptr<uint8_t[]> ok(new uint8_t[miss.size()]);
    base->PeekCoins(miss.data(), miss.size(), got.data(), ok.get());
    for (size_t k = 0; k < miss.size(); k++) {
        found[where[k]] = ok[k];
        if (ok[k]) coins[where[k]] = std::move(got[k]);
    }
}

bool CCoinsViewCache::HaveCoinInCache(const COutPoint& outpoint) const {
    auto it = cacheCoins.find(outpoint);
    return it != cacheCoins.end() && !it->second.coin.IsSpent();
}

uint256 CCoinsViewCache::GetBestBlock() const {
    if (hashBlock.IsNull()) hashBlock = base->GetBestBlock();
    return hashBlock;
}

void CCoinsViewCache::SetBestBlock(const uint256& h) { hashBlock = h; }

void CCoinsViewCache::ForEachShard(const std::function<void(unsigned)>& fn, WorkerPool* with) const {
    if (with) with->ParallelFor(CCoinsMap::SHARDS, [&](size_t s) { fn((unsigned)s); }, 1);
    else
        for (unsigned s = 0; s < CCoinsMap::SHARDS; s++) fn(s);
}

// a child's shard s into ours (the same s: the shard function is shared by every cache)
void CCoinsViewCache::MergeShard(CCoinsMap::Shard& from, unsigned s) {
    CCoinsMap::Shard& ours = cacheCoins.shard(s);
    size_t& used = usage[s].bytes;
    // the child's entries are left in place (moved-from) and freed with the child's map
    for (auto it = from.begin(); it != from.end(); ++it) {
        if (!(it->second.flags & CCoinsCacheEntry::DIRTY)) continue; // non-dirty: nothing to merge
        CCoinsMap::Shard::iterator itUs;
        if (it->second.flags & CCoinsCacheEntry::FRESH && it->second.coin.IsSpent()) {
            // created and spent in the child: nothing to add; only a spent parent copy matters
            itUs = ours.find(it->first);
            if (itUs == ours.end()) continue;
        } else {
            // one hash and probe for the common insert (a coin the block created)
            bool inserted;
            std::tie(itUs, inserted) = ours.try_emplace(it->first);
            if (inserted) {
                CCoinsCacheEntry& entry = itUs->second;
                entry.coin = std::move(it->second.coin);
                used += entry.coin.DynamicMemoryUsage();
                entry.flags = CCoinsCacheEntry::DIRTY;
                if (it->second.flags & CCoinsCacheEntry::FRESH) entry.flags |= CCoinsCacheEntry::FRESH;
                continue;
            }
        }
        {
            if ((it->second.flags & CCoinsCacheEntry::FRESH) && !itUs->second.coin.IsSpent())
                throw std::logic_error("FRESH flag misapplied to cache entry for base transaction with spendable outputs");
            if ((itUs->second.flags & CCoinsCacheEntry::FRESH) && it->second.coin.IsSpent()) {
                // parent entry is FRESH and now spent: forget it entirely
                used -= itUs->second.coin.DynamicMemoryUsage();
                ours.erase(itUs);
            } else {
                used -= itUs->second.coin.DynamicMemoryUsage();
                itUs->second.coin = std::move(it->second.coin);
                used += itUs->second.coin.DynamicMemoryUsage();
                itUs->second.flags |= CCoinsCacheEntry::DIRTY;
            }
        }
    }
}

bool CCoinsViewCache::BatchWrite(CCoinsMap& mapCoins, const uint256& hashBlockIn) {
    // a block's worth of entries merges one shard per task; a misapplied FRESH flag in any
    // shard is reported after every task has finished
    std::string err;
    std::mutex errMu;
    ForEachShard(
        [&](unsigned s) {
            try {
                MergeShard(mapCoins.shard(s), s);
            } catch (const std::logic_error& e) {
                std::lock_guard<std::mutex> l(errMu);
                err = e.what();
            }
        },
        mapCoins.size() >= 4096 ? pool : nullptr);
    if (!err.empty()) throw std::logic_error(err);
    hashBlock = hashBlockIn;
    return true;
}

bool CCoinsViewCache::Flush() {
    const bool ok = base->BatchWrite(cacheCoins, hashBlock);
    if (cacheCoins.size() >= 4096) {
        // a block's worth of merged-away entries (moved-from coins, ~80k nodes for an 8 MB
        // block) is freed on the reaper thread instead of the connecting one
        std::unique_ptr<CCoinsMap> dead(new CCoinsMap);
        dead->swap(cacheCoins);
        Reaper::Get().Drop(std::move(dead));
    } else {
        cacheCoins.clear();
    }
    for (ShardUsage& u : usage) u.bytes = 0;
    return ok;
}

void CCoinsViewCache::Uncache(const COutPoint& outpoint) {
    auto it = cacheCoins.find(outpoint);
    if (it != cacheCoins.end() && it->second.flags == 0) {
        usage[CCoinsMap::ShardOf(outpoint)].bytes -= it->second.coin.DynamicMemoryUsage();
        cacheCoins.erase(it);
    }
}

const CTxOut& CCoinsViewCache::GetOutputFor(const CTxIn& input) const {
    const Coin& c = AccessCoin(input.prevout);
    if (c.IsSpent()) throw std::logic_error("GetOutputFor on spent coin");
    return c.out;
}

Amount CCoinsViewCache::GetValueIn(const CTransaction& tx) const {
    if (tx.IsCoinBase()) return 0;
    Amount n = 0;
    for (const auto& in : tx.vin) n += GetOutputFor(in).nValue;
    return n;
}

bool CCoinsViewCache::HaveInputs(const CTransaction& tx) const {
    if (tx.IsCoinBase()) return true;
    for (const auto& in : tx.vin)
        if (!HaveCoin(in.prevout)) return false;
    return true;
}

static const size_t MAX_OUTPUTS_PER_TX = 1000000 / 9; // min txout size

const Coin& AccessByTxid(const CCoinsViewCache& view, const uint256& txid) {
    COutPoint iter(txid, 0);
    while (iter.n < MAX_OUTPUTS_PER_TX) {
        const Coin& alt = view.AccessCoin(iter);
        if (!alt.IsSpent()) return alt;
        ++iter.n;
    }
    return coinEmpty;
}

} // namespace bcp
