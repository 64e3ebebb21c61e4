// Embedded ordered key-value store (replaces the reference's LevelDB wrapper,
// src/dbwrapper.{h,cpp}: CDBWrapper Read/Write/Erase/Exists/WriteBatch/NewIterator,
// CDBBatch, EstimateSize, IsEmpty; used by src/txdb.cpp for the block index and UTXO set).
//
// Design: a single append-only log of CRC-protected batches plus an in-memory ordered
// index (key -> offset/length of the latest value in the log). Values are read back
// with pread, so memory holds keys only. A batch is durable once its record is written
// (optionally fsync'ed); a torn tail record is detected by the CRC on open and
// truncated, which gives the atomic-batch semantics the chainstate flush relies on.
// When dead bytes dominate the log it is rewritten (compaction) via write-new + rename.
#pragma once
#include "primitives/serialize.h"

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace bcp {

class KVStore;

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
    void WriteRaw(std::string key, std::string value) { ops.push_back({true, std::move(key), std::move(value)}); }
    void EraseRaw(std::string key) { ops.push_back({false, std::move(key), std::string()}); }
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

class KVIterator {
public:
    explicit KVIterator(const KVStore* db);
    void Seek(const std::string& rawKey);
    template <typename K> void Seek(const K& key) { Seek(KVBatch::Ser(key)); }
    void SeekToFirst();
    bool Valid() const { return valid; }
    void Next();
    const std::string& RawKey() const { return curKey; }
    bool RawValue(std::string& out) const;
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
        std::string raw;
        if (!RawValue(raw)) return false;
        try {
            SpanReader r((const unsigned char*)raw.data(), raw.size(), SER_DISK, PROTOCOL_VERSION);
            r >> value;
            return true;
        } catch (const std::exception&) {
            return false;
        }
    }

private:
    const KVStore* db;
    std::string curKey;
    bool valid = false;
};

class KVStore {
public:
    // path: directory; memory_only: no file backing (tests, -regtest in-memory dbs).
    KVStore(const std::string& path, bool memory_only = false, bool wipe = false);
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
    bool ReadRaw(const std::string& key, std::string& value) const;
    bool ExistsRaw(const std::string& key) const;
    bool IsEmpty() const;
    size_t Count() const;
    size_t EstimateSize(const std::string& begin, const std::string& end) const;
    std::unique_ptr<KVIterator> NewIterator() const { return std::unique_ptr<KVIterator>(new KVIterator(this)); }
    void Compact(); // rewrite the log with live records only
    uint64_t LogBytes() const { return logSize; }
    // Salvage (reference CDBEnv::Salvage / CWalletDB::Recover): scan a store's log without
    // trusting its structure — every batch whose header and CRC check out is replayed, damaged
    // stretches are skipped by searching for the next batch header (instead of truncating the
    // rest of the log as Replay does). Returns the latest value of every live key; `skipped`
    // counts the damaged bytes.
    static std::map<std::string, std::string> Salvage(const std::string& dir, uint64_t* skipped = nullptr);

private:
    friend class KVIterator;
    struct Loc {
        uint64_t off; // offset of the value bytes in the log (memory mode: index into mem)
        uint32_t len;
    };
    bool Replay();
    void MaybeCompact();
    void DoCompact();
    bool NextKey(const std::string& after, bool inclusive, std::string& out) const;

    std::string dir, logPath;
    bool memOnly;
    int fd = -1;
    uint64_t logSize = 0, liveBytes = 0;
    std::map<std::string, Loc> index;
    std::vector<std::string> mem; // memory-only value storage
    mutable std::mutex cs;
};

} // namespace bcp
