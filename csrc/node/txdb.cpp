#include "node/txdb.h"
#include "node/ui_interface.h"
#include "util/util.h"

#include "consensus/pow.h"
#include "util/strencodings.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

namespace bcp {

static BlockFileSizes g_fileSizes;
const BlockFileSizes& FileSizes() { return g_fileSizes; }
void SetFastPrune(bool on) {
    g_fileSizes = BlockFileSizes();
    if (on) {
        g_fileSizes.maxFile = 0x10000;
        g_fileSizes.blockChunk = 0x1000;
        g_fileSizes.undoChunk = 0x1000;
    }
}

namespace {
const char DB_COIN = 'C';
const char DB_BLOCK_FILES = 'f';
const char DB_TXINDEX = 't';
const char DB_BLOCK_INDEX = 'b';
const char DB_BEST_BLOCK = 'B';
const char DB_HEAD_BLOCKS = 'H';
const char DB_FLAG = 'F';
const char DB_REINDEX_FLAG = 'R';
const char DB_LAST_BLOCK = 'l';

// Coin key: 'C' || txid || VARINT(n) (reference txdb.cpp CoinEntry).
struct CoinKey {
    COutPoint* op;
    char key = DB_COIN;
    explicit CoinKey(const COutPoint* p) : op(const_cast<COutPoint*>(p)) {}
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, key);
        ::bcp::Serialize(s, op->hash);
        WriteVarInt(s, op->n);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, key);
        ::bcp::Unserialize(s, op->hash);
        op->n = (uint32_t)ReadVarInt(s);
    }
};
} // namespace

std::string CBlockFileInfo::ToString() const {
    return strprintf("CBlockFileInfo(blocks=%u, size=%u, heights=%u...%u)", nBlocks, nSize, nHeightFirst, nHeightLast);
}

// ------------------------------------------------------------------ coins db
// The reference gives LevelDB a quarter of the cache as write buffer and half as block cache
// (src/dbwrapper.cpp:72-80); the memtable and block cache here take the same shares.
static KVOptions CacheOptions(size_t nCacheSize) {
    KVOptions o;
    o.memtableBytes = std::max<size_t>(nCacheSize / 4, 1u << 20);
    o.blockCacheBytes = nCacheSize / 2;
    return o;
}

CCoinsViewDB::CCoinsViewDB(const std::string& dir, bool fMemory, bool fWipe, size_t nCacheSize)
    : db(dir, fMemory, fWipe, CacheOptions(nCacheSize)) {}

// Disk damage under the coin database (KVCorruption): the reference's CCoinsViewErrorCatcher
// (src/init.cpp:142-163) reports it and aborts. Returning false instead would read as a spent or
// missing coin, so ConnectBlock would reject a valid block and mark its chain invalid.
[[noreturn]] static void CoinsReadFailed(const std::exception& e) {
    uiInterface.ThreadSafeMessageBox("Error reading from database, shutting down.", "", CClientUIInterface::MSG_ERROR);
    LogPrintf("Error reading from database: %s\n", e.what());
    std::abort();
}

bool CCoinsViewDB::GetCoin(const COutPoint& outpoint, Coin& coin) const {
    try {
        return db.Read(CoinKey(&outpoint), coin);
    } catch (const KVCorruption& e) {
        CoinsReadFailed(e);
    }
}
bool CCoinsViewDB::HaveCoin(const COutPoint& outpoint) const {
    try {
        return db.Exists(CoinKey(&outpoint));
    } catch (const KVCorruption& e) {
        CoinsReadFailed(e);
    }
}

void CCoinsViewDB::PeekCoins(const COutPoint* outpoints, size_t n, Coin* coins, uint8_t* found) const {
    std::vector<std::string> keys(n), values(n);
    for (size_t i = 0; i < n; i++) keys[i] = KVBatch::Ser(CoinKey(&outpoints[i]));
    try {
        db.ReadRawMany(keys.data(), n, values.data(), found);
    } catch (const KVCorruption& e) {
        CoinsReadFailed(e);
    }
    for (size_t i = 0; i < n; i++) {
        if (!found[i]) continue;
        try {
            SpanReader r((const unsigned char*)values[i].data(), values[i].size(), SER_DISK, PROTOCOL_VERSION);
            r >> coins[i];
        } catch (const std::exception&) {
            found[i] = 0; // as Read() treats an undecodable value
        }
    }
}

uint256 CCoinsViewDB::GetBestBlock() const {
    uint256 h;
    if (!db.Read(DB_BEST_BLOCK, h)) return uint256();
    return h;
}

std::vector<uint256> CCoinsViewDB::GetHeadBlocks() const {
    std::vector<uint256> v;
    if (!db.Read(DB_HEAD_BLOCKS, v)) return {};
    return v;
}

bool CCoinsViewDB::BatchWrite(CCoinsMap& mapCoins, const uint256& hashBlock) {
    // Crash safety: first mark the flush as in progress (H = [new, old]), then write the
    // coins, then replace the marker by the new best block. On restart a remaining H
    // marker triggers a replay (see Chainstate::ReplayBlocks).
    KVBatch batch;
    uint256 old_tip = GetBestBlock();
    if (old_tip.IsNull()) {
        // a previous flush was interrupted (replay in progress): keep its base
        std::vector<uint256> heads = GetHeadBlocks();
        if (heads.size() == 2) old_tip = heads[1];
    }
    if (!hashBlock.IsNull()) {
        batch.Erase(DB_BEST_BLOCK);
        std::vector<uint256> heads{hashBlock, old_tip};
        batch.Write(DB_HEAD_BLOCKS, heads);
    }
    for (auto it = mapCoins.begin(); it != mapCoins.end(); it = mapCoins.erase(it)) {
        if (it->second.flags & CCoinsCacheEntry::DIRTY) {
            CoinKey k(&it->first);
            if (it->second.coin.IsSpent()) batch.Erase(k);
            else batch.Write(k, it->second.coin);
        }
        if (batch.SizeEstimate() > (16u << 20)) {
            if (!db.WriteBatch(batch)) return false;
        }
    }
    if (!hashBlock.IsNull()) {
        batch.Erase(DB_HEAD_BLOCKS);
        batch.Write(DB_BEST_BLOCK, hashBlock);
    }
    return db.WriteBatch(batch, true);
}

size_t CCoinsViewDB::EstimateSize() const {
    return db.EstimateSize(std::string(1, DB_COIN), std::string(1, (char)(DB_COIN + 1)));
}

namespace {
class CCoinsViewDBCursor : public CCoinsViewCursor {
public:
    CCoinsViewDBCursor(const KVStore& db, const uint256& best) : it(db.NewIterator()) {
        hashBlock = best;
        it->Seek(std::string(1, DB_COIN));
        Load();
    }
    bool GetKey(COutPoint& key) const override {
        if (!valid) return false;
        key = cur;
        return true;
    }
    bool GetValue(Coin& coin) const override { return valid && it->GetValue(coin); }
    bool Valid() const override { return valid; }
    void Next() override {
        it->Next();
        Load();
    }

private:
    void Load() {
        valid = false;
        if (!it->Valid() || it->RawKey().empty() || it->RawKey()[0] != DB_COIN) return;
        CoinKey k(&cur);
        valid = it->GetKey(k);
    }
    std::unique_ptr<KVIterator> it;
    COutPoint cur;
    bool valid = false;
};
} // namespace

std::unique_ptr<CCoinsViewCursor> CCoinsViewDB::Cursor() const {
    return std::unique_ptr<CCoinsViewCursor>(new CCoinsViewDBCursor(db, GetBestBlock()));
}

// ------------------------------------------------------------------ block tree db
CBlockTreeDB::CBlockTreeDB(const std::string& dir, bool fMemory, bool fWipe, size_t nCacheSize)
    : db(dir, fMemory, fWipe, CacheOptions(nCacheSize)) {}

bool CBlockTreeDB::WriteBatchSync(const std::vector<std::pair<int, const CBlockFileInfo*>>& fileInfo, int nLastFile,
                                  const std::vector<const CBlockIndex*>& blockinfo) {
    KVBatch batch;
    for (const auto& fi : fileInfo) batch.Write(std::make_pair(DB_BLOCK_FILES, fi.first), *fi.second);
    batch.Write(DB_LAST_BLOCK, nLastFile);
    for (const CBlockIndex* bi : blockinfo)
        batch.Write(std::make_pair(DB_BLOCK_INDEX, bi->GetBlockHash()), CDiskBlockIndex(bi));
    return db.WriteBatch(batch, true);
}

bool CBlockTreeDB::ReadBlockFileInfo(int nFile, CBlockFileInfo& info) {
    return db.Read(std::make_pair(DB_BLOCK_FILES, nFile), info);
}
bool CBlockTreeDB::ReadLastBlockFile(int& nFile) { return db.Read(DB_LAST_BLOCK, nFile); }
bool CBlockTreeDB::WriteReindexing(bool fReindexing) {
    if (fReindexing) return db.Write(DB_REINDEX_FLAG, '1');
    return db.Erase(DB_REINDEX_FLAG);
}
bool CBlockTreeDB::ReadReindexing(bool& fReindexing) {
    fReindexing = db.Exists(DB_REINDEX_FLAG);
    return true;
}
bool CBlockTreeDB::ReadTxIndex(const uint256& txid, CDiskTxPos& pos) {
    return db.Read(std::make_pair(DB_TXINDEX, txid), pos);
}
bool CBlockTreeDB::WriteTxIndex(const std::vector<std::pair<uint256, CDiskTxPos>>& list) {
    KVBatch batch;
    for (const auto& p : list) batch.Write(std::make_pair(DB_TXINDEX, p.first), p.second);
    return db.WriteBatch(batch);
}
bool CBlockTreeDB::WriteFlag(const std::string& name, bool fValue) {
    return db.Write(std::make_pair(DB_FLAG, name), fValue ? '1' : '0');
}
bool CBlockTreeDB::ReadFlag(const std::string& name, bool& fValue) {
    char ch;
    if (!db.Read(std::make_pair(DB_FLAG, name), ch)) return false;
    fValue = ch == '1';
    return true;
}

bool CBlockTreeDB::LoadBlockIndexGuts(const std::function<CBlockIndex*(const uint256&)>& insert,
                                      const Consensus::Params& params) {
    auto it = db.NewIterator();
    it->Seek(std::string(1, DB_BLOCK_INDEX));
    while (it->Valid()) {
        const std::string& k = it->RawKey();
        if (k.empty() || k[0] != DB_BLOCK_INDEX) break;
        CDiskBlockIndex disk;
        if (!it->GetValue(disk)) return false;
        const CBlockHeader hdr = disk.GetHeader();
        const uint256 hash = hdr.GetHash(params);
        CBlockIndex* pindex = insert(hash);
        pindex->pprev = insert(disk.hashPrev);
        pindex->nHeight = disk.nHeight;
        pindex->nFile = disk.nFile;
        pindex->nDataPos = disk.nDataPos;
        pindex->nUndoPos = disk.nUndoPos;
        pindex->nVersion = disk.nVersion;
        pindex->hashMerkleRoot = disk.hashMerkleRoot;
        memcpy(pindex->nReserved, disk.nReserved, sizeof(disk.nReserved));
        pindex->nTime = disk.nTime;
        pindex->nBits = disk.nBits;
        pindex->nNonce = disk.nNonce;
        pindex->nSolution = disk.nSolution;
        pindex->nStatus = disk.nStatus;
        pindex->nTx = disk.nTx;
        // header PoW re-check on load (reference txdb.cpp:261-266 checks SHA256d only)
        const bool postfork = (int)hdr.nHeight >= params.BCPHeight;
        if (!CheckProofOfWork(hash, pindex->nBits, postfork, params)) return false;
        it->Next();
    }
    return true;
}

// ------------------------------------------------------------------ flat files
static std::string g_blocksDir = "blocks";
void SetBlocksDir(const std::string& dir) {
    g_blocksDir = dir;
    ::mkdir(dir.c_str(), 0700);
}
const std::string& GetBlocksDir() { return g_blocksDir; }

std::string GetBlockPosFilename(const CDiskBlockPos& pos, const char* prefix) {
    return strprintf("%s/%s%05u.dat", g_blocksDir.c_str(), prefix, (unsigned)pos.nFile);
}

FILE* OpenDiskFile(const CDiskBlockPos& pos, const char* prefix, bool fReadOnly) {
    if (pos.IsNull()) return nullptr;
    const std::string path = GetBlockPosFilename(pos, prefix);
    FILE* f = fopen(path.c_str(), "rb+");
    if (!f && !fReadOnly) f = fopen(path.c_str(), "wb+");
    if (!f) return nullptr;
    if (pos.nPos && fseek(f, pos.nPos, SEEK_SET)) {
        fclose(f);
        return nullptr;
    }
    return f;
}

void AllocateFileRange(FILE* file, unsigned offset, unsigned length) {
    // posix_fallocate keeps block files contiguous; fall back to writing zeros
    const int fd = fileno(file);
    if (posix_fallocate(fd, offset, length) == 0) return;
    static const char buf[65536] = {};
    if (fseek(file, offset, SEEK_SET)) return;
    while (length > 0) {
        const unsigned now = std::min<unsigned>(sizeof(buf), length);
        fwrite(buf, 1, now, file);
        length -= now;
    }
}

namespace {
// stdio-backed stream adapter for the serializer
class FileStream {
public:
    FileStream(FILE* f, int type, int version) : f(f), nType(type), nVersion(version) {}
    ~FileStream() {
        if (f) fclose(f);
    }
    void write(const char* p, size_t n) {
        if (fwrite(p, 1, n, f) != n) throw std::ios_base::failure("FileStream::write: write failed");
    }
    void read(char* p, size_t n) {
        if (fread(p, 1, n, f) != n) throw std::ios_base::failure("FileStream::read: end of file");
    }
    int GetType() const { return nType; }
    int GetVersion() const { return nVersion; }
    FILE* Get() { return f; }
    template <typename T> FileStream& operator<<(const T& o) {
        ::bcp::Serialize(*this, o);
        return *this;
    }
    template <typename T> FileStream& operator>>(T& o) {
        ::bcp::Unserialize(*this, o);
        return *this;
    }

private:
    FILE* f;
    int nType, nVersion;
};
} // namespace

bool WriteBlockToDisk(const CBlock& block, CDiskBlockPos& pos, const unsigned char diskMagic[4]) {
    FileStream out(OpenBlockFile(pos), SER_DISK, PROTOCOL_VERSION);
    if (!out.Get()) return false;
    const uint32_t nSize = (uint32_t)GetSerializeSize(block, PROTOCOL_VERSION);
    out.write((const char*)diskMagic, 4);
    out << nSize;
    const long p = ftell(out.Get());
    if (p < 0) return false;
    pos.nPos = (unsigned)p;
    out << block;
    return true;
}

namespace {
// moves the reader past one serialized transaction (the layout CMutableTransaction::Unserialize
// reads, with the same compact-size range checks)
void SkipTransaction(SpanReader& r) {
    r.ignore(4); // nVersion
    const uint64_t nIn = ReadCompactSize(r);
    for (uint64_t i = 0; i < nIn; i++) {
        r.ignore(36); // prevout
        r.ignore(ReadCompactSize(r)); // scriptSig
        r.ignore(4); // nSequence
    }
    const uint64_t nOut = ReadCompactSize(r);
    for (uint64_t i = 0; i < nOut; i++) {
        r.ignore(8); // nValue
        r.ignore(ReadCompactSize(r)); // scriptPubKey
    }
    r.ignore(4); // nLockTime
}
} // namespace

bool DecodeBlock(const unsigned char* data, size_t len, CBlock& block, WorkerPool* pool) {
    block.SetNull();
    try {
        SpanReader r(data, len, SER_DISK, PROTOCOL_VERSION);
        static_cast<CBlockHeader&>(block).Unserialize(r);
        const uint64_t ntx = ReadCompactSize(r);
        if (ntx > len / 10) return false; // not even 10 bytes per transaction: truncated or corrupt
        if (!pool || ntx < 256) {
            block.vtx.reserve(ntx);
            for (uint64_t i = 0; i < ntx; i++) block.vtx.push_back(std::make_shared<const CTransaction>(deserialize, r));
            return true;
        }
        // one pass finds every transaction's bytes, then they are decoded (and their txids
        // hashed) in parallel
        std::vector<size_t> start(ntx + 1);
        for (uint64_t i = 0; i < ntx; i++) {
            start[i] = r.tell();
            SkipTransaction(r);
        }
        start[ntx] = r.tell();
        block.vtx.resize(ntx);
        std::atomic<bool> bad{false};
        pool->ParallelFor(
            ntx,
            [&](size_t i) {
                try {
                    SpanReader tr(data + start[i], start[i + 1] - start[i], SER_DISK, PROTOCOL_VERSION);
                    block.vtx[i] = std::make_shared<const CTransaction>(deserialize, tr);
                    if (!tr.empty()) bad = true;
                } catch (const std::exception&) {
                    bad = true;
                }
            },
            32);
        if (bad) block.SetNull();
        return !bad;
    } catch (const std::exception&) {
        block.SetNull();
        return false;
    }
}

bool ReadBlockFromDisk(CBlock& block, const CDiskBlockPos& pos, const CChainParams& params, bool checkPow,
                       WorkerPool* pool) {
    block.SetNull();
    std::vector<unsigned char> raw;
    if (pool && ReadRawBlockFromDisk(raw, pos)) {
        // the whole record in one read, decoded in memory (the stream path below reads field by field)
        if (!DecodeBlock(raw.data(), raw.size(), block, pool)) return false;
    } else {
        FileStream in(OpenBlockFile(pos, true), SER_DISK, PROTOCOL_VERSION);
        if (!in.Get()) return false;
        try {
            in >> block;
        } catch (const std::exception&) {
            return false;
        }
    }
    if (!checkPow) return true;
    const bool postfork = (int)block.nHeight >= params.GetConsensus().BCPHeight;
    if (postfork && !CheckEquihashSolution(&block, params)) return false;
    return CheckProofOfWork(block.GetHash(params.GetConsensus()), block.nBits, postfork, params.GetConsensus());
}

bool ReadBlockFromDisk(CBlock& block, const CBlockIndex* pindex, const CChainParams& params, bool checkPow,
                       WorkerPool* pool) {
    if (!ReadBlockFromDisk(block, pindex->GetBlockPos(), params, checkPow, pool)) return false;
    return block.GetHash(params.GetConsensus()) == pindex->GetBlockHash();
}

bool ReadRawBlockFromDisk(std::vector<unsigned char>& out, const CDiskBlockPos& pos) {
    if (pos.nPos < 8) return false;
    CDiskBlockPos hpos(pos.nFile, pos.nPos - 8);
    FILE* f = OpenBlockFile(hpos, true);
    if (!f) return false;
    unsigned char hdr[8];
    bool ok = fread(hdr, 1, 8, f) == 8;
    uint32_t size = 0;
    if (ok) {
        memcpy(&size, hdr + 4, 4);
        out.resize(size);
        ok = size < (64u << 20) && fread(out.data(), 1, size, f) == size;
    }
    fclose(f);
    return ok;
}

uint256 UndoChecksum(const std::vector<unsigned char>& ser, const uint256& hashBlock) {
    HashWriter hasher;
    hasher << hashBlock;
    hasher.write((const char*)ser.data(), ser.size());
    return hasher.GetHash();
}

bool UndoWriteToDisk(const std::vector<unsigned char>& ser, CDiskBlockPos& pos, const uint256& hashBlock,
                     const unsigned char diskMagic[4], const uint256* checksum) {
    // one serialisation, one hash pass and one write: the undo record is serialised once by the
    // caller (the reference serialises it three times - size, file, checksum - through small
    // buffered writes). The checksum is SHA256d(hashBlock || record), as the reference's.
    FileStream out(OpenUndoFile(pos), SER_DISK, PROTOCOL_VERSION);
    if (!out.Get()) return false;
    const uint32_t nSize = (uint32_t)ser.size();
    out.write((const char*)diskMagic, 4);
    out << nSize;
    const long p = ftell(out.Get());
    if (p < 0) return false;
    pos.nPos = (unsigned)p;
    out.write((const char*)ser.data(), ser.size());
    out << (checksum ? *checksum : UndoChecksum(ser, hashBlock));
    return true;
}

bool UndoWriteToDisk(const CBlockUndo& undo, CDiskBlockPos& pos, const uint256& hashBlock,
                     const unsigned char diskMagic[4]) {
    return UndoWriteToDisk(SerializeToBytes(undo, SER_DISK, PROTOCOL_VERSION), pos, hashBlock, diskMagic);
}

bool UndoReadFromDisk(CBlockUndo& undo, const CDiskBlockPos& pos, const uint256& hashBlock) {
    FileStream in(OpenUndoFile(pos, true), SER_DISK, PROTOCOL_VERSION);
    if (!in.Get()) return false;
    uint256 checksum;
    try {
        in >> undo;
        in >> checksum;
    } catch (const std::exception&) {
        return false;
    }
    HashWriter hasher;
    hasher << hashBlock << undo;
    return checksum == hasher.GetHash();
}

} // namespace bcp
