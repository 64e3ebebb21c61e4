// Embedded ordered key-value store (replaces the reference's LevelDB wrapper,
// src/dbwrapper.{h,cpp}: CDBWrapper Read/Write/Erase/Exists/WriteBatch/NewIterator,
// CDBBatch, EstimateSize, IsEmpty; used by src/txdb.cpp for the block index and UTXO set,
// and by the wallet).
//
// Design: a log-structured merge store whose memory is bounded by its options, not by the
// number of keys.
//  * Writes append one CRC-protected record per batch to the write-ahead log (kv-<n>.log) and
//    apply the batch to an in-memory ordered table (the memtable). A batch is atomic: on open,
//    a torn or corrupt tail record is dropped and the log truncated there.
//  * When the memtable passes `memtableBytes` (or its log passes twice that) it becomes
//    immutable, a new log starts, and a background thread writes it out as a sorted segment
//    (seg-<n>.sst: CRC'd data blocks, a sparse block index and a Bloom filter). Writers only
//    wait if a second memtable fills before the first is on disk.
//  * Segments are immutable. The background thread merges runs of adjacent segments when there
//    are more than `maxSegments` (tombstones are dropped when the run reaches the oldest
//    segment); readers and iterators keep the segment set they started with (shared
//    ownership), so a merge never blocks them and never pulls a file out from under them.
//  * MANIFEST (written to a temporary file, fsync'ed, renamed) names the live segments and the
//    first log still needed; files it does not name are deleted on open.
//  * Memory: the memtable(s), per segment a sparse index (one key per ~blockSize bytes) and a
//    Bloom filter (bloomBitsPerKey bits per key), and an LRU cache of decoded blocks
//    (blockCacheBytes). Point reads cost at most one block read per segment whose filter
//    matches.
// A pre-segment store (a single kv.log of batch records) is read as a log and migrated on open.
#pragma once
#include "primitives/serialize.h"

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace bcp {

class KVStore;

// A stored block that fails its CRC or cannot be read (disk damage).
struct KVCorruption : std::runtime_error {
    using std::runtime_error::runtime_error;
};

class KVBatch {
public:
    template <typename K, typename V> void Write(const K& key, const V& value) {
        ops.push_back({true, Ser(key), Ser(value)});
        bytes += ops.back().key.size() + ops.back().value.size();
    }
    template <typename K> void Erase(const K& key) {
        ops.push_back({false, Ser(key), std::string()});
        bytes += ops.back().key.size();
    }
    void WriteRaw(std::string key, std::string value) {
        bytes += key.size() + value.size();
        ops.push_back({true, std::move(key), std::move(value)});
    }
    void EraseRaw(std::string key) {
        bytes += key.size();
        ops.push_back({false, std::move(key), std::string()});
    }
    size_t SizeEstimate() const { return bytes; }
    void Clear() {
        ops.clear();
        bytes = 0;
    }
    bool Empty() const { return ops.empty(); }

    template <typename T> static std::string Ser(const T& t) {
        std::vector<unsigned char> v;
        VectorWriter w(v, SER_DISK, PROTOCOL_VERSION);
        w << t;
        return std::string(v.begin(), v.end());
    }

private:
    friend class KVStore;
    struct Op {
        bool put;
        std::string key, value;
    };
    std::vector<Op> ops;
    size_t bytes = 0;
};

// Ordered iteration over a consistent set of segments plus the live memtable (writes made
// while iterating may or may not be seen, as with the reference's LevelDB iterators).
class KVIterator {
public:
    explicit KVIterator(const KVStore* db);
    ~KVIterator();
    void Seek(const std::string& rawKey);
    template <typename K> void Seek(const K& key) { Seek(KVBatch::Ser(key)); }
    void SeekToFirst();
    bool Valid() const { return valid; }
    void Next();
    const std::string& RawKey() const { return curKey; }
    bool RawValue(std::string& out) const {
        if (!valid) return false;
        out = curValue;
        return true;
    }
    template <typename K> bool GetKey(K& key) const {
        try {
            SpanReader r((const unsigned char*)curKey.data(), curKey.size(), SER_DISK, PROTOCOL_VERSION);
            r >> key;
            return true;
        } catch (const std::exception&) {
            return false;
        }
    }
    template <typename V> bool GetValue(V& value) const {
        if (!valid) return false;
        try {
            SpanReader r((const unsigned char*)curValue.data(), curValue.size(), SER_DISK, PROTOCOL_VERSION);
            r >> value;
            return true;
        } catch (const std::exception&) {
            return false;
        }
    }

    struct State;

private:
    void Settle(); // move to the first live entry at or after the sources' positions
    const KVStore* db;
    std::unique_ptr<State> st;
    std::string curKey, curValue;
    bool valid = false;
};

struct KVOptions {
    size_t memtableBytes = 64u << 20;   // memtable size that triggers a segment flush
    size_t blockCacheBytes = 32u << 20; // decoded-block LRU cache
    size_t blockBytes = 4u << 10;       // target data block size
    int bloomBitsPerKey = 10;           // ~1% false positives
    int maxSegments = 8;                // more segments than this start a background merge
    int mergeWidth = 4;                 // segments merged at once
};

struct KVStats {
    size_t segments = 0;
    uint64_t segmentBytes = 0, logBytes = 0;
    size_t memtableBytes = 0, immutableBytes = 0;
    size_t indexBytes = 0, bloomBytes = 0, cacheBytes = 0;
    uint64_t flushes = 0, merges = 0, stalls = 0, bloomSkips = 0, blockReads = 0;
};

class KVStore {
public:
    // path: directory; memory_only: no file backing (tests, -regtest in-memory dbs).
    KVStore(const std::string& path, bool memory_only = false, bool wipe = false, const KVOptions& opts = KVOptions());
    ~KVStore();
    KVStore(const KVStore&) = delete;

    template <typename K, typename V> bool Read(const K& key, V& value) const {
        std::string raw;
        if (!ReadRaw(KVBatch::Ser(key), raw)) return false;
        try {
            SpanReader r((const unsigned char*)raw.data(), raw.size(), SER_DISK, PROTOCOL_VERSION);
            r >> value;
        } catch (const std::exception&) {
            return false;
        }
        return true;
    }
    template <typename K, typename V> bool Write(const K& key, const V& value, bool fSync = false) {
        KVBatch b;
        b.Write(key, value);
        return WriteBatch(b, fSync);
    }
    template <typename K> bool Exists(const K& key) const { return ExistsRaw(KVBatch::Ser(key)); }
    template <typename K> bool Erase(const K& key, bool fSync = false) {
        KVBatch b;
        b.Erase(key);
        return WriteBatch(b, fSync);
    }
    bool WriteBatch(KVBatch& batch, bool fSync = false);
    // A missing key reads as false; a segment block that fails its CRC or cannot be read throws
    // KVCorruption (the reference's dbwrapper_error, src/dbwrapper.cpp HandleError): disk damage
    // must never look like an absent key.
    bool ReadRaw(const std::string& key, std::string& value) const;
    // ReadRaw of n keys under one acquisition of the store lock (batched lookups from many
    // threads would otherwise contend on it per key): found[i] says whether values[i] is set.
    void ReadRawMany(const std::string* keys, size_t n, std::string* values, uint8_t* found) const;
    bool ExistsRaw(const std::string& key) const;
    bool IsEmpty() const;
    size_t Count() const; // live keys (a full scan)
    size_t EstimateSize(const std::string& begin, const std::string& end) const;
    std::unique_ptr<KVIterator> NewIterator() const { return std::unique_ptr<KVIterator>(new KVIterator(this)); }
    // Flush the memtable and merge every segment into one (tombstones dropped); synchronous.
    void Compact();
    // Write the memtable out as a segment now and wait for it (tests, shutdown paths).
    void Flush();
    uint64_t LogBytes() const; // bytes on disk (logs + segments)
    KVStats Stats() const;
    // Salvage (reference CDBEnv::Salvage / CWalletDB::Recover): read a store's files without
    // trusting its manifest — every segment block and log batch whose CRC checks out is kept,
    // damaged stretches are skipped (log batches by searching for the next record header).
    // Returns the latest value of every live key; `skipped` counts the damaged bytes.
    static std::map<std::string, std::string> Salvage(const std::string& dir, uint64_t* skipped = nullptr);
    // Fault injection (tests): the next manifest write / segment write fails.
    enum : int { FAULT_MANIFEST = 1, FAULT_SEGMENT = 2 };
    void InjectFault(int what);

    struct Impl;

private:
    friend class KVIterator;
    std::unique_ptr<Impl> d;
};

} // namespace bcp
