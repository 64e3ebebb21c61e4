// UTXO set: Coin, compressed on-disk encoding, layered coin views and the cache.
// Parity: reference src/coins.{h,cpp} (Coin :27-70 height<<1|coinbase, CCoinsView,
// CCoinsViewBacked, CCoinsViewCache with DIRTY/FRESH flags, BatchWrite, AddCoins,
// SpendCoin with undo capture, AccessByTxid) and src/compressor.{h,cpp}
// (CompressAmount/DecompressAmount, 6 special script encodings), src/undo.h
// (CTxUndo/CBlockUndo, TxInUndoSerializer).
#pragma once
#include "crypto/hashes.h"
#include "primitives/transaction.h"
#include "util/poolalloc.h"
#include "util/util.h"

#include <functional>
#include <memory>
#include <type_traits>
#include <unordered_map>

namespace bcp {

uint64_t CompressAmount(uint64_t n);
uint64_t DecompressAmount(uint64_t x);

// Script compression: P2PKH/P2SH/P2PK stored in 21 or 33 bytes.
bool CompressScript(const CScript& script, std::vector<unsigned char>& out);
unsigned GetSpecialScriptSize(unsigned nSize);
bool DecompressScript(CScript& script, unsigned nSize, const std::vector<unsigned char>& in);
static const unsigned int nSpecialScripts = 6;

template <typename S> void SerializeCompressedScript(S& s, const CScript& script) {
    std::vector<unsigned char> compr;
    if (CompressScript(script, compr)) {
        s.write((const char*)compr.data(), compr.size());
        return;
    }
    WriteVarInt(s, script.size() + nSpecialScripts);
    s.write((const char*)script.data(), script.size());
}
template <typename S> void UnserializeCompressedScript(S& s, CScript& script) {
    uint64_t nSize = ReadVarInt(s);
    if (nSize < nSpecialScripts) {
        std::vector<unsigned char> v(GetSpecialScriptSize((unsigned)nSize));
        s.read((char*)v.data(), v.size());
        DecompressScript(script, (unsigned)nSize, v);
        return;
    }
    nSize -= nSpecialScripts;
    if (nSize > (unsigned)MAX_SCRIPT_SIZE) {
        // overly long script: replace with a short unspendable one, skip the payload
        script.clear();
        script << OP_RETURN;
        char skip[4096]; // in chunks: a bogus multi-GB size hits the end of the stream, not the allocator
        for (uint64_t left = nSize; left > 0;) {
            const size_t k = (size_t)std::min<uint64_t>(left, sizeof(skip));
            s.read(skip, k);
            left -= k;
        }
    } else {
        script.resize(nSize);
        s.read((char*)script.data(), nSize);
    }
}
template <typename S> void SerializeCompressedTxOut(S& s, const CTxOut& out) {
    WriteVarInt(s, CompressAmount((uint64_t)out.nValue));
    SerializeCompressedScript(s, out.scriptPubKey);
}
template <typename S> void UnserializeCompressedTxOut(S& s, CTxOut& out) {
    out.nValue = (Amount)DecompressAmount(ReadVarInt(s));
    UnserializeCompressedScript(s, out.scriptPubKey);
}

class Coin {
public:
    CTxOut out;
    bool fCoinBase = false;
    uint32_t nHeight = 0;

    Coin() {}
    Coin(CTxOut o, int h, bool cb) : out(std::move(o)), fCoinBase(cb), nHeight((uint32_t)h) {}
    void Clear() {
        out.SetNull();
        CScript().swap(out.scriptPubKey); // release the script's buffer: a spent entry costs no usage
        fCoinBase = false;
        nHeight = 0;
    }
    bool IsSpent() const { return out.IsNull(); }
    bool IsCoinBase() const { return fCoinBase; }
    uint32_t GetHeight() const { return nHeight; }
    const CTxOut& GetTxOut() const { return out; }
    // the script's heap block, if it has one (scripts of up to 28 bytes live inside the Coin)
    size_t DynamicMemoryUsage() const {
        const size_t a = out.scriptPubKey.allocated_memory();
        return a ? ((a + 8 + 15) & ~(size_t)15) : 0;
    }

    template <typename S> void Serialize(S& s) const {
        WriteVarInt(s, (uint64_t)nHeight * 2 + (fCoinBase ? 1 : 0));
        SerializeCompressedTxOut(s, out);
    }
    template <typename S> void Unserialize(S& s) {
        const uint64_t code = ReadVarInt(s);
        nHeight = (uint32_t)(code >> 1);
        fCoinBase = code & 1;
        UnserializeCompressedTxOut(s, out);
    }
};

// Undo record of one spent input: the coin, with height/coinbase always present
// (format is the reference's post-0.15 TxInUndoSerializer: VARINT(h*2+cb), [VARINT(0)
// if h>0], compressed txout).
struct TxInUndoFormatter {
    template <typename S> static void Ser(S& s, const Coin& c) {
        WriteVarInt(s, (uint64_t)c.nHeight * 2 + (c.fCoinBase ? 1 : 0));
        if (c.nHeight > 0) WriteVarInt(s, 0); // legacy tx-version placeholder
        SerializeCompressedTxOut(s, c.out);
    }
    template <typename S> static void Unser(S& s, Coin& c) {
        const uint64_t code = ReadVarInt(s);
        c.nHeight = (uint32_t)(code >> 1);
        c.fCoinBase = code & 1;
        if (c.nHeight > 0) ReadVarInt(s);
        UnserializeCompressedTxOut(s, c.out);
    }
};

class CTxUndo {
public:
    std::vector<Coin> vprevout;
    template <typename S> void Serialize(S& s) const {
        WriteCompactSize(s, vprevout.size());
        for (const Coin& c : vprevout) TxInUndoFormatter::Ser(s, c);
    }
    template <typename S> void Unserialize(S& s) {
        const uint64_t n = ReadCompactSize(s);
        if (n > MAX_TX_SIZE_FOR_UNDO) throw ser_error("too many input undo records");
        vprevout.resize(n);
        for (Coin& c : vprevout) TxInUndoFormatter::Unser(s, c);
    }
    static const uint64_t MAX_TX_SIZE_FOR_UNDO = 1000000 / 41; // min txin size
};

class CBlockUndo {
public:
    std::vector<CTxUndo> vtxundo; // one per tx except the coinbase
    template <typename S> void Serialize(S& s) const { ::bcp::Serialize(s, vtxundo); }
    template <typename S> void Unserialize(S& s) { ::bcp::Unserialize(s, vtxundo); }
};

struct SaltedOutpointHasher {
    uint64_t k0, k1;
    SaltedOutpointHasher();
    size_t operator()(const COutPoint& o) const { return SipHashUint256Extra(k0, k1, o.hash.begin(), o.n); }
};

struct CCoinsCacheEntry {
    Coin coin;
    unsigned char flags = 0;
    enum Flags { DIRTY = 1, FRESH = 2 };
    CCoinsCacheEntry() {}
    explicit CCoinsCacheEntry(Coin&& c) : coin(std::move(c)) {}
};
// A coins cache's entries, split over SHARDS hash maps by a fixed function of the outpoint (the
// reference's single CCoinsMap, src/coins.h:183). Because the split is the same in every cache,
// a child's shard i only ever merges into its parent's shard i, and the entries of one shard
// never touch another's: a block's view updates and the flush of a block's view into the tip
// run one shard per thread. Each shard is salted-SipHash keyed (collision flooding stays as hard
// as in the reference) and takes its nodes from its own arena (util/poolalloc.h).
class CCoinsMap {
public:
    static constexpr unsigned SHARDS = 16;
    typedef std::unordered_map<COutPoint, CCoinsCacheEntry, SaltedOutpointHasher, std::equal_to<COutPoint>,
                               NodePoolAllocator<std::pair<const COutPoint, CCoinsCacheEntry>>>
        Shard;
    typedef Shard::value_type value_type;

    // txids are already uniform hashes: the top bits of a cheap mix choose the shard
    static unsigned ShardOf(const COutPoint& o) {
        return (unsigned)((o.hash.GetCheapHash() + (uint64_t)o.n * 0x9E3779B97F4A7C15ULL) >> 60);
    }

    template <bool Const> class Iter {
    public:
        typedef std::conditional_t<Const, const CCoinsMap, CCoinsMap> Map;
        typedef std::conditional_t<Const, Shard::const_iterator, Shard::iterator> Inner;
        typedef std::conditional_t<Const, const Shard::value_type, Shard::value_type> Value;
        typedef std::forward_iterator_tag iterator_category;
        typedef std::ptrdiff_t difference_type;
        typedef Value value_type;
        typedef Value* pointer;
        typedef Value& reference;

        Iter() = default;
        Iter(Map* m, unsigned s, Inner i) : map(m), shard(s), it(i) { Settle(); }
        template <bool C, typename = std::enable_if_t<Const && !C>>
        Iter(const Iter<C>& o) : map(o.map), shard(o.shard), it(o.it) {}
        Value& operator*() const { return *it; }
        Value* operator->() const { return &*it; }
        Iter& operator++() {
            ++it;
            Settle();
            return *this;
        }
        bool operator==(const Iter& o) const { return shard == o.shard && it == o.it; }
        bool operator!=(const Iter& o) const { return !(*this == o); }

    private:
        template <bool> friend class Iter;
        friend class CCoinsMap;
        // past the end of a shard: move to the next non-empty one (the last shard's end is end())
        void Settle() {
            while (it == map->shards[shard].end() && shard + 1 < SHARDS) it = map->shards[++shard].begin();
        }
        Map* map = nullptr;
        unsigned shard = 0;
        Inner it;
    };
    typedef Iter<false> iterator;
    typedef Iter<true> const_iterator;

    iterator begin() { return iterator(this, 0, shards[0].begin()); }
    iterator end() { return iterator(this, SHARDS - 1, shards[SHARDS - 1].end()); }
    const_iterator begin() const { return const_iterator(this, 0, shards[0].begin()); }
    const_iterator end() const { return const_iterator(this, SHARDS - 1, shards[SHARDS - 1].end()); }
    iterator find(const COutPoint& k) {
        const unsigned s = ShardOf(k);
        auto it = shards[s].find(k);
        return it == shards[s].end() ? end() : iterator(this, s, it);
    }
    const_iterator find(const COutPoint& k) const {
        const unsigned s = ShardOf(k);
        auto it = shards[s].find(k);
        return it == shards[s].end() ? end() : const_iterator(this, s, it);
    }
    iterator erase(iterator pos) { return iterator(this, pos.shard, shards[pos.shard].erase(pos.it)); }
    CCoinsCacheEntry& operator[](const COutPoint& k) { return shards[ShardOf(k)][k]; }
    size_t size() const {
        size_t n = 0;
        for (const Shard& s : shards) n += s.size();
        return n;
    }
    bool empty() const { return size() == 0; }
    // Empties every shard and hands its node arena back to the system: the shard is swapped
    // with a fresh one (the allocators travel with the swap), so the old arena's chunks go
    // with the temporary instead of staying behind as free-list slack.
    void clear() {
        for (Shard& s : shards) {
            Shard fresh;
            s.swap(fresh);
        }
    }
    // exchanges every shard (and its arena) with o's
    void swap(CCoinsMap& o) {
        for (unsigned i = 0; i < SHARDS; i++) shards[i].swap(o.shards[i]);
    }
    // room for n entries spread over the shards (with slack for an uneven split)
    void reserve(size_t n) {
        for (Shard& s : shards) s.reserve(n / SHARDS + n / (4 * SHARDS) + 16);
    }
    size_t bucket_count() const {
        size_t n = 0;
        for (const Shard& s : shards) n += s.bucket_count();
        return n;
    }
    Shard& shard(unsigned i) { return shards[i]; }
    const Shard& shard(unsigned i) const { return shards[i]; }

private:
    Shard shards[SHARDS];
};

class CCoinsViewCursor {
public:
    virtual ~CCoinsViewCursor() {}
    virtual bool GetKey(COutPoint& key) const = 0;
    virtual bool GetValue(Coin& coin) const = 0;
    virtual bool Valid() const = 0;
    virtual void Next() = 0;
    const uint256& GetBestBlock() const { return hashBlock; }

protected:
    uint256 hashBlock;
};

class CCoinsView {
public:
    virtual ~CCoinsView() {}
    virtual bool GetCoin(const COutPoint& outpoint, Coin& coin) const { return false; }
    virtual bool HaveCoin(const COutPoint& outpoint) const {
        Coin c;
        return GetCoin(outpoint, c);
    }
    virtual uint256 GetBestBlock() const { return uint256(); }
    virtual bool BatchWrite(CCoinsMap& mapCoins, const uint256& hashBlock) { return false; }
    virtual std::unique_ptr<CCoinsViewCursor> Cursor() const { return nullptr; }
    virtual size_t EstimateSize() const { return 0; }
    // GetCoin without filling any cache on the way, so several threads may peek at once while
    // nobody writes (the database view's reads are thread-safe; caches override this).
    virtual bool PeekCoin(const COutPoint& outpoint, Coin& coin) const { return GetCoin(outpoint, coin); }
    // PeekCoin of n outpoints at once (the database answers a batch under one lock).
    virtual void PeekCoins(const COutPoint* outpoints, size_t n, Coin* coins, uint8_t* found) const {
        for (size_t i = 0; i < n; i++) found[i] = PeekCoin(outpoints[i], coins[i]);
    }
};

class CCoinsViewBacked : public CCoinsView {
public:
    explicit CCoinsViewBacked(CCoinsView* v) : base(v) {}
    bool GetCoin(const COutPoint& o, Coin& c) const override { return base->GetCoin(o, c); }
    bool HaveCoin(const COutPoint& o) const override { return base->HaveCoin(o); }
    uint256 GetBestBlock() const override { return base->GetBestBlock(); }
    bool BatchWrite(CCoinsMap& m, const uint256& h) override { return base->BatchWrite(m, h); }
    std::unique_ptr<CCoinsViewCursor> Cursor() const override { return base->Cursor(); }
    size_t EstimateSize() const override { return base->EstimateSize(); }
    void SetBackend(CCoinsView& v) { base = &v; }

protected:
    CCoinsView* base;
};

class CCoinsViewCache : public CCoinsViewBacked {
public:
    explicit CCoinsViewCache(CCoinsView* base);
    CCoinsViewCache(const CCoinsViewCache&) = delete;

    bool GetCoin(const COutPoint& outpoint, Coin& coin) const override;
    bool HaveCoin(const COutPoint& outpoint) const override;
    uint256 GetBestBlock() const override;
    void SetBestBlock(const uint256& hashBlock);
    bool BatchWrite(CCoinsMap& mapCoins, const uint256& hashBlock) override;
    std::unique_ptr<CCoinsViewCursor> Cursor() const override {
        throw std::logic_error("CCoinsViewCache cursor iteration not supported");
    }

    bool PeekCoin(const COutPoint& outpoint, Coin& coin) const override;
    void PeekCoins(const COutPoint* outpoints, size_t n, Coin* coins, uint8_t* found) const override;
    bool HaveCoinInCache(const COutPoint& outpoint) const;
    const Coin& AccessCoin(const COutPoint& output) const;
    // This cache's own entry for an outpoint (spent or not), without asking the base.
    const Coin* FindInCache(const COutPoint& outpoint) const {
        auto it = cacheCoins.find(outpoint);
        return it == cacheCoins.end() ? nullptr : &it->second.coin;
    }
    // SpendCoin of an unspent coin this cache does not hold yet, given the base's copy of it
    // (read through PeekCoin while the stack below was as it is now): the same entry FetchCoin
    // followed by SpendCoin would leave, without the round trip through the base.
    void SpendFetched(const COutPoint& outpoint, Coin&& coin, Coin* moveto);
    // The same entry when the caller already moved the base's copy of the coin elsewhere (into
    // an undo record): a spent, DIRTY, not FRESH entry.
    void SpendFetchedMoved(const COutPoint& outpoint);
    // Spends an unspent coin the caller read through PeekCoins and already moved elsewhere (into
    // an undo record), whether or not this cache holds it: its own entry is erased when FRESH and
    // otherwise left spent and DIRTY (SpendCoin); with no entry, a spent, DIRTY, not FRESH one is
    // added (SpendFetchedMoved). Never reads the base. Safe under ForEachShard.
    void SpendPeeked(const COutPoint& outpoint);
    void AddCoin(const COutPoint& outpoint, Coin&& coin, bool possible_overwrite);
    bool SpendCoin(const COutPoint& outpoint, Coin* moveto = nullptr);
    bool Flush();
    void Uncache(const COutPoint& outpoint);
    unsigned int GetCacheSize() const { return (unsigned)cacheCoins.size(); }
    // Sizes the entry table for n entries up front (a block connect knows how many it adds).
    void Reserve(size_t n) { cacheCoins.reserve(n); }
    size_t BucketCount() const { return cacheCoins.bucket_count(); }
    size_t DynamicMemoryUsage() const;
    Amount GetValueIn(const CTransaction& tx) const;
    bool HaveInputs(const CTransaction& tx) const;
    const CTxOut& GetOutputFor(const CTxIn& input) const;
    // A pool for shard-parallel work: a large BatchWrite into this cache merges one shard per
    // task. The cache is still single-writer: the pool only splits that one call.
    void SetPool(WorkerPool* p) { pool = p; }
    // Calls fn(shard) for every shard, on the pool when one is set; fn may only touch entries of
    // its own shard (AddCoin / SpendCoin / SpendFetchedMoved of outpoints in it, and SpendCoin
    // only of entries this cache already holds).
    void ForEachShard(const std::function<void(unsigned)>& fn, WorkerPool* with) const;

protected:
    CCoinsMap::iterator FetchCoin(const COutPoint& outpoint) const;
    // bytes of the coins' own heap buffers, per shard (one cache line each)
    struct alignas(64) ShardUsage {
        size_t bytes = 0;
    };
    size_t CachedCoinsUsage() const {
        size_t n = 0;
        for (const ShardUsage& u : usage) n += u.bytes;
        return n;
    }
    void MergeShard(CCoinsMap::Shard& from, unsigned s);
    mutable uint256 hashBlock;
    mutable CCoinsMap cacheCoins;
    mutable ShardUsage usage[CCoinsMap::SHARDS];
    WorkerPool* pool = nullptr;
};

// Add all outputs of a tx. check=true handles the BIP30 overwrite case.
void AddCoins(CCoinsViewCache& cache, const CTransaction& tx, int nHeight, bool check = false);
const Coin& AccessByTxid(const CCoinsViewCache& cache, const uint256& txid);

} // namespace bcp
