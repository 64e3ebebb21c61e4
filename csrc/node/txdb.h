// Persistent chainstate databases and flat block files.
// Parity: reference src/txdb.{h,cpp} (key prefixes C/B/H coins, b/f/l/R/F/t block
// tree, CCoinsViewDB::BatchWrite with head-blocks crash marker, LoadBlockIndexGuts),
// src/chain.h CBlockFileInfo, src/validation.cpp WriteBlockToDisk :1096,
// ReadBlockFromDisk :1120 (re-checks Equihash + PoW), UndoWriteToDisk :1521,
// UndoReadFromDisk :1547 (checksum = SHA256d(prev hash || undo)).
#pragma once
#include "consensus/chain.h"
#include "consensus/params.h"
#include "node/coins.h"
#include "node/kvstore.h"

#include <functional>
#include <string>

namespace bcp {
class WorkerPool;

struct CBlockFileInfo {
    unsigned nBlocks = 0, nSize = 0, nUndoSize = 0, nHeightFirst = 0, nHeightLast = 0;
    uint64_t nTimeFirst = 0, nTimeLast = 0;
    template <typename S> void Serialize(S& s) const {
        WriteVarInt(s, nBlocks);
        WriteVarInt(s, nSize);
        WriteVarInt(s, nUndoSize);
        WriteVarInt(s, nHeightFirst);
        WriteVarInt(s, nHeightLast);
        WriteVarInt(s, nTimeFirst);
        WriteVarInt(s, nTimeLast);
    }
    template <typename S> void Unserialize(S& s) {
        nBlocks = (unsigned)ReadVarInt(s);
        nSize = (unsigned)ReadVarInt(s);
        nUndoSize = (unsigned)ReadVarInt(s);
        nHeightFirst = (unsigned)ReadVarInt(s);
        nHeightLast = (unsigned)ReadVarInt(s);
        nTimeFirst = ReadVarInt(s);
        nTimeLast = ReadVarInt(s);
    }
    void AddBlock(unsigned nHeightIn, uint64_t nTimeIn) {
        if (nBlocks == 0 || nHeightFirst > nHeightIn) nHeightFirst = nHeightIn;
        if (nBlocks == 0 || nTimeFirst > nTimeIn) nTimeFirst = nTimeIn;
        nBlocks++;
        if (nHeightIn > nHeightLast) nHeightLast = nHeightIn;
        if (nTimeIn > nTimeLast) nTimeLast = nTimeIn;
    }
    std::string ToString() const;
};

struct CDiskTxPos : public CDiskBlockPos {
    unsigned nTxOffset = 0; // after the header
    CDiskTxPos() {}
    CDiskTxPos(const CDiskBlockPos& b, unsigned off) : CDiskBlockPos(b), nTxOffset(off) {}
    template <typename S> void Serialize(S& s) const {
        CDiskBlockPos::Serialize(s);
        WriteVarInt(s, nTxOffset);
    }
    template <typename S> void Unserialize(S& s) {
        CDiskBlockPos::Unserialize(s);
        nTxOffset = (unsigned)ReadVarInt(s);
    }
};

class CCoinsViewDB : public CCoinsView {
public:
    // nCacheSize: the store's memory budget (memtable + block cache), reference txdb.cpp:68
    CCoinsViewDB(const std::string& dir, bool fMemory, bool fWipe, size_t nCacheSize = 8u << 20);
    bool GetCoin(const COutPoint& outpoint, Coin& coin) const override;
    bool HaveCoin(const COutPoint& outpoint) const override;
    void PeekCoins(const COutPoint* outpoints, size_t n, Coin* coins, uint8_t* found) const override;
    uint256 GetBestBlock() const override;
    std::vector<uint256> GetHeadBlocks() const;
    bool BatchWrite(CCoinsMap& mapCoins, const uint256& hashBlock) override;
    std::unique_ptr<CCoinsViewCursor> Cursor() const override;
    size_t EstimateSize() const override;
    KVStore& DB() { return db; }

private:
    KVStore db;
};

class CBlockTreeDB {
public:
    CBlockTreeDB(const std::string& dir, bool fMemory, bool fWipe, size_t nCacheSize = 2u << 20);
    bool WriteBatchSync(const std::vector<std::pair<int, const CBlockFileInfo*>>& fileInfo, int nLastFile,
                        const std::vector<const CBlockIndex*>& blockinfo);
    bool ReadBlockFileInfo(int nFile, CBlockFileInfo& info);
    bool ReadLastBlockFile(int& nFile);
    bool WriteReindexing(bool fReindex);
    bool ReadReindexing(bool& fReindex);
    bool ReadTxIndex(const uint256& txid, CDiskTxPos& pos);
    bool WriteTxIndex(const std::vector<std::pair<uint256, CDiskTxPos>>& list);
    bool WriteFlag(const std::string& name, bool fValue);
    bool ReadFlag(const std::string& name, bool& fValue);
    // Rebuilds the in-memory block index; insert(hash) returns the (possibly new) entry.
    bool LoadBlockIndexGuts(const std::function<CBlockIndex*(const uint256&)>& insert,
                            const Consensus::Params& params);

private:
    KVStore db;
};

// ---- flat files (blocks/blkNNNNN.dat, blocks/revNNNNN.dat)
static const unsigned int MAX_BLOCKFILE_SIZE = 0x8000000; // 128 MiB
static const unsigned int BLOCKFILE_CHUNK_SIZE = 0x1000000; // 16 MiB
static const unsigned int UNDOFILE_CHUNK_SIZE = 0x100000;  // 1 MiB
// -fastprune (regtest): 64 KiB block files and 4 KiB preallocation chunks, so tests can fill,
// prune and reload many files with a short chain (later reference releases' option of that name)
struct BlockFileSizes {
    unsigned maxFile = MAX_BLOCKFILE_SIZE, blockChunk = BLOCKFILE_CHUNK_SIZE, undoChunk = UNDOFILE_CHUNK_SIZE;
};
const BlockFileSizes& FileSizes();
void SetFastPrune(bool on);

void SetBlocksDir(const std::string& dir);
const std::string& GetBlocksDir();
std::string GetBlockPosFilename(const CDiskBlockPos& pos, const char* prefix);
FILE* OpenDiskFile(const CDiskBlockPos& pos, const char* prefix, bool fReadOnly);
inline FILE* OpenBlockFile(const CDiskBlockPos& pos, bool ro = false) { return OpenDiskFile(pos, "blk", ro); }
inline FILE* OpenUndoFile(const CDiskBlockPos& pos, bool ro = false) { return OpenDiskFile(pos, "rev", ro); }
void AllocateFileRange(FILE* file, unsigned offset, unsigned length);

bool WriteBlockToDisk(const CBlock& block, CDiskBlockPos& pos, const unsigned char diskMagic[4]);
// Reads the raw block; `checkPow` re-validates Equihash/PoW like the reference.
// With a pool, the record is read in one piece and its transactions decoded in parallel
// (DecodeBlock); without one, field by field from the file.
bool ReadBlockFromDisk(CBlock& block, const CDiskBlockPos& pos, const CChainParams& params, bool checkPow = true,
                       WorkerPool* pool = nullptr);
bool ReadBlockFromDisk(CBlock& block, const CBlockIndex* pindex, const CChainParams& params, bool checkPow = true,
                       WorkerPool* pool = nullptr);
// Decodes a serialized block (disk format). With a pool and 256+ transactions, one pass finds
// the transactions' boundaries and they are decoded - txids hashed - in parallel. Any decode
// error (truncation, trailing bytes inside a transaction's span) fails the whole block.
bool DecodeBlock(const unsigned char* data, size_t len, CBlock& block, WorkerPool* pool);
bool ReadRawBlockFromDisk(std::vector<unsigned char>& out, const CDiskBlockPos& pos);
// the same for an already serialised (SER_DISK) undo record; `checksum`, when given, is its
// UndoChecksum (computed off the caller's critical path)
bool UndoWriteToDisk(const std::vector<unsigned char>& ser, CDiskBlockPos& pos, const uint256& hashBlock,
                     const unsigned char diskMagic[4], const uint256* checksum = nullptr);
// SHA256d(hashBlock || record): the checksum stored after an undo record
uint256 UndoChecksum(const std::vector<unsigned char>& ser, const uint256& hashBlock);
bool UndoWriteToDisk(const CBlockUndo& undo, CDiskBlockPos& pos, const uint256& hashBlock,
                     const unsigned char diskMagic[4]);
bool UndoReadFromDisk(CBlockUndo& undo, const CDiskBlockPos& pos, const uint256& hashBlock);

} // namespace bcp
